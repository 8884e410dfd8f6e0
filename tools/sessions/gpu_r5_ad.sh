#!/bin/bash
# Round 5 (ad): long context under planner off - window / run-ahead sweep vs static.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('link_gbps_per_gpu'), a.get('ring_per_step'), {k: (a.get('stream_stats_per_step') or {}).get(k) for k in ('prefetch_ms','ahead_wait_ms','wait_ms','use_ms')})"; }
lc() {
  local tag=$1; shift
  env "$@" timeout -k 10 700 python -u bench.py --no-aux --context 32768 --batch 8 --kv-tiering --steps 3 --warmup 2 > gpurun_out/r5/ad_$tag.log 2>&1 || { echo LC_FAIL $tag; tail -30 gpurun_out/r5/ad_$tag.log; return 1; }
  summ gpurun_out/r5/ad_$tag.log $tag
}
lc win4g_ahead64 OGKM_WINDOW_MB=4096 OGKM_MAX_AHEAD=64 && lc win8g_ahead64 OGKM_WINDOW_MB=8192 OGKM_MAX_AHEAD=64 && lc win8g OGKM_WINDOW_MB=8192 || exit 1
echo ALL_OK
