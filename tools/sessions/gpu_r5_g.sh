#!/bin/bash
# Round 5 (g): attention P.V with more V loads in flight (numerics + shapes),
# config 2 planner off vs static after the lease / hint batching, 70B headline.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused.py > gpurun_out/r5/g_fused.log 2>&1 || { echo FUSED_FAIL; tail -30 gpurun_out/r5/g_fused.log; exit 1; }
tail -2 gpurun_out/r5/g_fused.log
for d in 0 4 8; do
  env OGKM_ATTN_DPL=$d timeout -k 10 300 python -u tools/bench_attn.py > gpurun_out/r5/g_attn_dpl$d.log 2>&1 || { echo ATTN_FAIL $d; tail -20 gpurun_out/r5/g_attn_dpl$d.log; exit 1; }
  echo "== dpl $d"; cat gpurun_out/r5/g_attn_dpl$d.log
done
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a['traffic_per_step_gb']['pcie_measured'], a.get('stream_stats_per_step'))"; }
run_b() {  # $1 = tag, rest = bench args
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py --no-aux "$@" > gpurun_out/r5/g_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/g_$tag.log; return 1; }
  summ gpurun_out/r5/g_$tag.log $tag
}
run_b c2_off --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b 70b --steps 6 --warmup 4 && \
run_b tp8sim --simulate-tp 8 --steps 8 --warmup 3 || exit 1
echo ALL_OK
