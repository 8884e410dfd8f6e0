#!/bin/bash
# GPU tests (optional: SKIP_TESTS=1) + one 70B bench run with ${BENCH_ARGS}; each step time-limited.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head -30; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
timeout -k 10 450 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
