#!/bin/bash
# Round 5 (af): shards read duplicates on the GPU (2-rank test), long context with
# the 16-unit default window (twice), transparent 70B on this build.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_tp2.py > gpurun_out/r5/af_tp2.log 2>&1 || { echo TP2_FAIL; tail -30 gpurun_out/r5/af_tp2.log; exit 1; }
grep -E "max \||passed" gpurun_out/r5/af_tp2.log
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('link_gbps_per_gpu'), a.get('ring_per_step'), {k: (a.get('stream_stats_per_step') or {}).get(k) for k in ('prefetch_ms','ahead_wait_ms','wait_ms','use_ms')})"; }
for t in a b; do
  timeout -k 10 700 python -u bench.py --no-aux --context 32768 --batch 8 --kv-tiering --steps 3 --warmup 2 > gpurun_out/r5/af_lc_$t.log 2>&1 || { echo LC_FAIL; tail -30 gpurun_out/r5/af_lc_$t.log; exit 1; }
  summ gpurun_out/r5/af_lc_$t.log lc_$t
done
echo ALL_OK
