#!/bin/bash
# Round-3 check: GPU suite, smoke, 70B headline, the stock-torch managed-mode
# bench (8B, 2x oversubscribed), the HBM<->NUMA-node path probe, and the decode
# GEMM microbench (fused vs split-K) under rocprofv3. Each step time-limited;
# stop at the first failure.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
bash tools/gpu_verify.sh || exit 1
timeout -k 10 180 ./tools/bin/probe_cxl_paths 1024 > gpurun_out/r3/cxl_paths.jsonl 2> gpurun_out/r3/cxl_paths.err || { echo PROBE_FAIL; tail -5 gpurun_out/r3/cxl_paths.err; exit 1; }
wc -l gpurun_out/r3/cxl_paths.jsonl
SHAPES="6144x4096,4096x4096,28672x4096,4096x14336" VARIANTS="fused:2,raw:2" timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/dgemm8b.jsonl 2> gpurun_out/r3/dgemm8b.err || { echo DG8_FAIL; tail -20 gpurun_out/r3/dgemm8b.err; exit 1; }
cat gpurun_out/r3/dgemm8b.jsonl
VARIANTS="fused:2,raw:2" timeout -k 10 300 python -u tools/bench_dgemm.py > gpurun_out/r3/dgemm70b.jsonl 2> gpurun_out/r3/dgemm70b.err || { echo DG70_FAIL; tail -20 gpurun_out/r3/dgemm70b.err; exit 1; }
cat gpurun_out/r3/dgemm70b.jsonl
timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r3/tm8b.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r3/tm8b.log; exit 1; }
grep '^{' gpurun_out/r3/tm8b.log | cut -c1-1500
timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 10 --warmup 3 --no-aux > gpurun_out/r3/config2.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/config2.log; exit 1; }
grep '^{' gpurun_out/r3/config2.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_c2 -o run -- python bench.py --model llama3-8b --oversub 1 --steps 5 --warmup 2 --no-aux > gpurun_out/r3/prof_c2.log 2>&1 || { echo PROF_C2_FAIL; tail -20 gpurun_out/r3/prof_c2.log; exit 1; }
echo ALL_OK
