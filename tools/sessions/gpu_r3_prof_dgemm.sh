#!/bin/bash
# Kernel trace of the decode GEMM microbench (8B shapes, pipelined split-K):
# per-kernel durations of k_dgemm_pipe and k_dgemm_reduce.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
S8="6144x4096,4096x4096,28672x4096,4096x14336"
SHAPES=$S8 VARIANTS="raw:2" OGKM_DGEMM_LDS=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_dg8 -o run -- python tools/bench_dgemm.py > gpurun_out/r3/prof_dg8.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/prof_dg8.log; exit 1; }
VARIANTS="raw:2" OGKM_DGEMM_LDS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_dg70 -o run -- python tools/bench_dgemm.py > gpurun_out/r3/prof_dg70.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/prof_dg70.log; exit 1; }
timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 2 --warmup 1 > gpurun_out/r3/tm_a.log 2>&1; grep '^{' gpurun_out/r3/tm_a.log | cut -c 1-1200
OGKM_MANAGED_LOOKAHEAD_MB=0 timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 2 --warmup 1 > gpurun_out/r3/tm_b.log 2>&1; grep '^{' gpurun_out/r3/tm_b.log | cut -c 1-1200
OGKM_MANAGED_MIN_MB=64 timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 2 --warmup 1 > gpurun_out/r3/tm_c.log 2>&1; grep '^{' gpurun_out/r3/tm_c.log | cut -c 1-1200
echo ALL_OK
