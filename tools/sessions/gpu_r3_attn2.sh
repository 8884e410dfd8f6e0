#!/bin/bash
# Adaptive attention split (64-token one-wave workgroups on small grids): numerics, cold-KV bench.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_fused.py tests/test_dgemm.py tests/test_model_gpu.py > gpurun_out/r3/attn2_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r3/attn2_tests.log; exit 1; }
tail -2 gpurun_out/r3/attn2_tests.log
for S in 256 64 0; do
  SPLIT=$S timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/r3/attn2_$S.txt 2>&1 || { echo BA_FAIL; tail -20 gpurun_out/r3/attn2_$S.txt; exit 1; }
  grep GB/s gpurun_out/r3/attn2_$S.txt
done

for R in 1 2; do
  timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/c2_attn2_$R.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/c2_attn2_$R.log; exit 1; }
  echo "c2 $(grep '^{' gpurun_out/r3/c2_attn2_$R.log | cut -c1-150)"
done

timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3/h70_attn2.log 2>&1 || { echo H70_FAIL; tail -30 gpurun_out/r3/h70_attn2.log; exit 1; }
echo "70b $(grep '^{' gpurun_out/r3/h70_attn2.log | cut -c1-200)"
echo ALL_OK
