#!/bin/bash
# Round 5 (c): runtime-decided spread classes (SpreadPolicy) - headline with no
# model-side classes vs the policy off; the stock-torch 70B / 8B under
# ogkm.managed() with and without it; the 2-rank GPU tests under the default
# planner (shards now hinted too).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['config']['planner'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux'].get('stream_stats_per_step'), d['aux'].get('ring_per_step'))"; }
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 500 python -u bench.py --torch-managed --model $model --oversub 2 --steps 3 --warmup 3 > gpurun_out/r5/c_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/c_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/c_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
}
timeout -k 10 400 python -u bench.py --steps 6 --warmup 4 --no-aux > gpurun_out/r5/c_70b.log 2>&1 || { echo RUN_FAIL 70b; tail -30 gpurun_out/r5/c_70b.log; exit 1; }
summ gpurun_out/r5/c_70b.log 70b_runtime_spread
env RT_PERF_SPREAD_ENABLE=0 timeout -k 10 400 python -u bench.py --steps 6 --warmup 4 --no-aux > gpurun_out/r5/c_70b_nospread.log 2>&1 || { echo RUN_FAIL 70b_nospread; tail -30 gpurun_out/r5/c_70b_nospread.log; exit 1; }
summ gpurun_out/r5/c_70b_nospread.log 70b_belady_only
run_tm 70b_spread llama3-70b X=1 && run_tm 70b_nospread llama3-70b RT_PERF_SPREAD_ENABLE=0 || exit 1
run_tm 8b_spread llama3-8b X=1 && run_tm 8b_nospread llama3-8b RT_PERF_SPREAD_ENABLE=0 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tp2.py > gpurun_out/r5/c_tp2.log 2>&1; rc=$?
tail -4 gpurun_out/r5/c_tp2.log
exit $rc
