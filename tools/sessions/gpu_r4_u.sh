#!/bin/bash
# Round 4: config-2 timed-step kernel trace (one-launch norm), PMC (FETCH_SIZE, TA_BUSY) on the decode GEMM and
# attention microbenchmarks at the 8B shapes, 70B headline timed-step kernel trace.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
rm -rf gpurun_out/r4/prof_c2c gpurun_out/r4/pmc_gemm gpurun_out/r4/pmc_attn gpurun_out/r4/prof_70b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_c2c -o run -- python bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r4/u_c2.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r4/u_c2.log; exit 1; }
grep '^{' gpurun_out/r4/u_c2.log | cut -c1-200
SHAPES=6144x4096,4096x4096,28672x4096,4096x14336 VARIANTS=pipe:0 COLD=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr -d gpurun_out/r4/pmc_gemm -o pmc -- python tools/bench_dgemm.py > gpurun_out/r4/u_pmc_gemm.log 2>&1 || { echo PMC_GEMM_FAIL; tail -20 gpurun_out/r4/u_pmc_gemm.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4/pmc_gemm --filter dgemm > gpurun_out/r4/u_pmc_gemm.txt 2>&1; head -20 gpurun_out/r4/u_pmc_gemm.txt
ITERS=3 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr -d gpurun_out/r4/pmc_attn -o pmc -- python tools/bench_attn.py > gpurun_out/r4/u_pmc_attn.log 2>&1 || { echo PMC_ATTN_FAIL; tail -20 gpurun_out/r4/u_pmc_attn.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4/pmc_attn --filter attn > gpurun_out/r4/u_pmc_attn.txt 2>&1; head -20 gpurun_out/r4/u_pmc_attn.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_70b -o run -- python bench.py --steps 6 --warmup 3 --no-aux > gpurun_out/r4/u_70b.log 2>&1 || { echo PROF70_FAIL; tail -20 gpurun_out/r4/u_70b.log; exit 1; }
grep '^{' gpurun_out/r4/u_70b.log | cut -c1-200
echo ALL_OK
