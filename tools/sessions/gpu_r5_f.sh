#!/bin/bash
# Round 5 (f): resident-extent lease fast path - config 2 planner off (no fallback)
# vs static on the same box, the 70B headline, tp8-shard sim, stock-torch 8B/70B.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a['traffic_per_step_gb']['pcie_measured'], a.get('stream_stats_per_step'), a.get('ring_per_step'), {k: a.get('spread', {}).get(k) for k in ('keep_fraction', 'last_pass_keep_evictions')})"; }
run_b() {  # $1 = tag, rest = bench args
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py --no-aux "$@" > gpurun_out/r5/f_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/f_$tag.log; return 1; }
  summ gpurun_out/r5/f_$tag.log $tag
}
run_tm() {  # $1 = tag, $2 = model
  timeout -k 10 500 python -u bench.py --torch-managed --model $2 --oversub 2 --steps 3 --warmup 3 > gpurun_out/r5/f_tm_$1.log 2>&1 || { echo TM_FAIL $1; tail -30 gpurun_out/r5/f_tm_$1.log; return 1; }
  grep '^{' gpurun_out/r5/f_tm_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm_$1', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
}
run_b c2_off --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b c2_off_b --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b 70b --steps 6 --warmup 4 && \
run_b tp8sim --simulate-tp 8 --steps 8 --warmup 3 && \
run_tm 8b llama3-8b && run_tm 70b llama3-70b || exit 1
echo ALL_OK
