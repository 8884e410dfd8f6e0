#!/bin/bash
# Config 2 (Llama-3-8B, HBM-resident, bf16) decode: host enqueue vs GPU step
# time, per-kernel trace of the bench, and the 8B decode-GEMM shapes alone.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 240 python -u tools/prof_host_step.py --model llama3-8b --simulate-tp 1 --oversub 1 --steps 10 \
  --weight-format bf16 --kv-format bf16 > gpurun_out/r3/host_c2.txt 2>&1 || { echo HOST_FAIL; tail -20 gpurun_out/r3/host_c2.txt; exit 1; }
head -4 gpurun_out/r3/host_c2.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_c2b -o run -- python bench.py --model llama3-8b --oversub 1 --steps 10 --warmup 3 --no-aux > gpurun_out/r3/prof_c2b.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/prof_c2b.log; exit 1; }
grep '^{' gpurun_out/r3/prof_c2b.log | cut -c1-200
SHAPES="6144x4096,4096x4096,28672x4096,4096x14336" VARIANTS="raw:2" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_dg8b -o run -- python tools/bench_dgemm.py > gpurun_out/r3/prof_dg8b.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/prof_dg8b.log; exit 1; }
grep '^{' gpurun_out/r3/prof_dg8b.log | cut -c1-400
echo ALL_OK
