#!/bin/bash
# Auto pipe / LDS-ring decode GEMM plan: numerics + model tests, per-shape sweep
# (auto vs k_dgemm_pipe), config 2 (Llama-3-8B HBM-resident) bench.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dgemm.py tests/test_model_gpu.py tests/test_fused.py > gpurun_out/r3/auto_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r3/auto_tests.log; exit 1; }
tail -2 gpurun_out/r3/auto_tests.log
grep "layer total" gpurun_out/r3/auto_tests.log || true
S8="6144x4096,4096x4096,28672x4096,4096x14336,128256x4096"
SHAPES=$S8 VARIANTS="pipe:0,pipe:4" timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/auto8b.jsonl 2>&1 || { echo B8_FAIL; tail -20 gpurun_out/r3/auto8b.jsonl; exit 1; }
VARIANTS="pipe:0,pipe:4" timeout -k 10 300 python -u tools/bench_dgemm.py > gpurun_out/r3/auto70b.jsonl 2>&1 || { echo B70_FAIL; tail -20 gpurun_out/r3/auto70b.jsonl; exit 1; }
grep '^{' gpurun_out/r3/auto8b.jsonl | cut -c1-360; grep '^{' gpurun_out/r3/auto70b.jsonl | cut -c1-360
timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 10 --warmup 3 --no-aux > gpurun_out/r3/config2_auto.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/config2_auto.log; exit 1; }
grep '^{' gpurun_out/r3/config2_auto.log | cut -c1-300
echo ALL_OK
