#!/bin/bash
# Quick GPU verification: GPU tests, smoke, 70B bench. Each step time-limited; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo GPU_TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 450 python bench.py --steps 5 --warmup 2 > gpurun_out/bench70b.log 2>&1 || { echo B70_FAIL; tail -30 gpurun_out/bench70b.log; exit 1; }
grep '^{' gpurun_out/bench70b.log
