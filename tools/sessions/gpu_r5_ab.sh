#!/bin/bash
# Round 5 (ab): long-context (32k, batch 8, KV tiered) under planner off was 8.1
# tok/s vs 11.2 static in round 2 - A/B: static, a longer run-ahead, the Python
# unit protocol; then the transparent 70B block census.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('link_gbps_per_gpu'), a.get('ring_per_step'), {k: (a.get('stream_stats_per_step') or {}).get(k) for k in ('prefetch_ms','ahead_wait_ms','wait_ms','use_ms')})"; }
lc() {
  local tag=$1; shift
  env "${@:2}" timeout -k 10 700 python -u bench.py --no-aux --context 32768 --batch 8 --kv-tiering --steps 3 --warmup 2 $1 > gpurun_out/r5/ab_$tag.log 2>&1 || { echo LC_FAIL $tag; tail -30 gpurun_out/r5/ab_$tag.log; return 1; }
  summ gpurun_out/r5/ab_$tag.log $tag
}
lc static "--planner static" X=1 && lc ahead64 "" OGKM_MAX_AHEAD=64 && lc pyunits "" OGKM_NATIVE_UNITS=0 || exit 1
OGKM_TM_CENSUS=1 OGKM_PACK=1 timeout -k 10 700 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 3 > gpurun_out/r5/ab_tm_census.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r5/ab_tm_census.log; exit 1; }
grep '^{' gpurun_out/r5/ab_tm_census.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step']); print(json.dumps(a['block_census'], indent=1)); print(a['pack'])"
echo ALL_OK
