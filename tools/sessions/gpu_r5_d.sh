#!/bin/bash
# Round 5 (d): headline with exact runtime spread classes; stock-torch 8B A/B of
# the two new ring / arena behaviours (the transparent mode slowed in (c)).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux'].get('ring_per_step'), d['aux'].get('spread'))"; }
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 500 python -u bench.py --torch-managed --model $model --oversub 2 --steps 3 --warmup 3 > gpurun_out/r5/d_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/d_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/d_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'], a.get('spread'))"
}
timeout -k 10 400 python -u bench.py --steps 6 --warmup 4 --no-aux > gpurun_out/r5/d_70b.log 2>&1 || { echo RUN_FAIL 70b; tail -30 gpurun_out/r5/d_70b.log; exit 1; }
summ gpurun_out/r5/d_70b.log 70b_runtime_spread
run_tm 8b_default llama3-8b X=1 || exit 1
run_tm 8b_nowaitissued llama3-8b RT_RING_WAIT_ISSUED=0 || exit 1
run_tm 8b_norerank llama3-8b RT_ARENA_VICTIM_RERANK=0 || exit 1
run_tm 8b_neither llama3-8b RT_RING_WAIT_ISSUED=0 RT_ARENA_VICTIM_RERANK=0 RT_PERF_SPREAD_ENABLE=0 || exit 1
echo ALL_OK
