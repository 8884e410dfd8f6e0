#!/bin/bash
# Round 5 (h): native unit protocol - GPU model numerics, 2-rank tests, config 2
# planner off vs static, 70B headline, tp8 sim, 405B tp8 sim.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_gpu_tp2.py tests/test_fused.py > gpurun_out/r5/h_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/r5/h_tests.log; exit 1; }
tail -2 gpurun_out/r5/h_tests.log
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a['traffic_per_step_gb']['pcie_measured'], a.get('stream_stats_per_step'))"; }
run_b() {  # $1 = tag, rest = bench args
  local tag=$1; shift
  timeout -k 10 500 python -u bench.py --no-aux "$@" > gpurun_out/r5/h_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/h_$tag.log; return 1; }
  summ gpurun_out/r5/h_$tag.log $tag
}
run_b c2_off --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b 70b --steps 6 --warmup 4 && \
run_b tp8sim --simulate-tp 8 --steps 8 --warmup 3 && \
run_b 405tp8 --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 6 --warmup 3 || exit 1
echo ALL_OK
