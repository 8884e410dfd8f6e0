#!/bin/bash
# Round 5 (ao): tp8 shard simulations on the final tree (70B; 405B three tiers).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; s=a.get('stream_stats_per_step') or {}; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], {k: s.get(k) for k in ('prefetch_ms','acquire_ms','use_ms')})"; }
timeout -k 10 600 python -u bench.py --no-aux --simulate-tp 8 --steps 8 --warmup 3 > gpurun_out/r5/ao_tp8sim.log 2>&1 || { echo TP8_FAIL; tail -30 gpurun_out/r5/ao_tp8sim.log; exit 1; }
summ gpurun_out/r5/ao_tp8sim.log tp8sim
timeout -k 10 700 python -u bench.py --no-aux --model llama3-405b --tiers host+cxl --simulate-tp 8 --steps 4 --warmup 2 > gpurun_out/r5/ao_405tp8.log 2>&1 || { echo T405_FAIL; tail -30 gpurun_out/r5/ao_405tp8.log; exit 1; }
summ gpurun_out/r5/ao_405tp8.log 405tp8
echo ALL_OK
