#!/bin/bash
# Multi-workgroup RMSNorm (+ deferred residual): numerics, config 2 twice, and a
# kernel trace of config 2's timed steps.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fused.py tests/test_model_gpu.py > gpurun_out/r3/norm_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r3/norm_tests.log; exit 1; }
tail -2 gpurun_out/r3/norm_tests.log
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/c2_norm_$R.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/c2_norm_$R.log; exit 1; }
  echo "c2 $(grep '^{' gpurun_out/r3/c2_norm_$R.log | cut -c1-150)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_c2e -o run -- python bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/prof_c2e.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/prof_c2e.log; exit 1; }
echo ALL_OK
