#!/bin/bash
# Round 4 final (2): the tp2 GPU test alone, then the rest of the GPU suite, smoke, headline bench (planner off
# default) and the static plan.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_tp2.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/final_tp2.log 2>&1; echo "tp2 rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r4/final_tp2.log | head -5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --deselect tests/test_gpu_tp2.py::test_two_ranks_match_fp32_reference[tp] --deselect tests/test_gpu_tp2.py::test_two_ranks_match_fp32_reference[shards] > gpurun_out/r4/final_gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|ERROR" gpurun_out/r4/final_gpu_tests.log | head -20; tail -20 gpurun_out/r4/final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4/final_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/final_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r4/final_smoke.log; exit 1; }
tail -1 gpurun_out/r4/final_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4/final_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r4/final_bench.log; exit 1; }
grep '^{' gpurun_out/r4/final_bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py --planner static > gpurun_out/r4/final_bench_static.log 2>&1 || { echo STATIC_FAIL; tail -20 gpurun_out/r4/final_bench_static.log; exit 1; }
grep '^{' gpurun_out/r4/final_bench_static.log | cut -c1-200
echo ALL_OK
