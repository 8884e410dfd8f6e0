#!/bin/bash
# Round 4 last check: transparent-mode / allocator GPU tests, smoke, headline bench, stock-torch 8B.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_managed_mode_gpu.py tests/test_gpu_tp2.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/last_tests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/r4/last_tests.log; exit 1; }
tail -1 gpurun_out/r4/last_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/last_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r4/last_smoke.log; exit 1; }
tail -1 gpurun_out/r4/last_smoke.log | cut -c1-80
timeout -k 10 400 python -u bench.py > gpurun_out/r4/last_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r4/last_bench.log; exit 1; }
grep '^{' gpurun_out/r4/last_bench.log | cut -c1-200
timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r4/last_tm8.log 2>&1 || { echo TM_FAIL; tail -20 gpurun_out/r4/last_tm8.log; exit 1; }
grep '^{' gpurun_out/r4/last_tm8.log | cut -c1-200
echo ALL_OK
