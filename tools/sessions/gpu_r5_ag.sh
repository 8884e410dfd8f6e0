#!/bin/bash
# Round 5 (ag): host cost of next-use victim searches - long context (13-unit
# window) and the headline.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('link_gbps_per_gpu'), a.get('ring_per_step'), {k: (a.get('stream_stats_per_step') or {}).get(k) for k in ('prefetch_ms','ahead_wait_ms','wait_ms','use_ms')})"; }
timeout -k 10 700 python -u bench.py --no-aux --context 32768 --batch 8 --kv-tiering --steps 3 --warmup 2 > gpurun_out/r5/ag_lc.log 2>&1 || { echo LC_FAIL; tail -30 gpurun_out/r5/ag_lc.log; exit 1; }
summ gpurun_out/r5/ag_lc.log lc
timeout -k 10 700 python -u bench.py --no-aux --steps 6 --warmup 3 > gpurun_out/r5/ag_70b.log 2>&1 || { echo HL_FAIL; tail -30 gpurun_out/r5/ag_70b.log; exit 1; }
summ gpurun_out/r5/ag_70b.log 70b
echo ALL_OK
