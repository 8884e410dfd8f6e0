#!/bin/bash
# Round 5 (a): tp8-shard simulation under planner off vs static (host cost per
# unit), then the 2-rank peer-shard run under planner off (the round-4 hang)
# with the launcher's SIGUSR1 stack + runtime dumps.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['config']['planner'], d['aux']['traffic_per_step_gb'], d['aux'].get('stream_stats_per_step'), d['aux'].get('ring_per_step'))"; }
for pl in off static; do
  timeout -k 10 400 python -u bench.py --simulate-tp 8 --planner $pl --steps 8 --warmup 3 --no-aux > gpurun_out/r5/a_tp8sim_$pl.log 2>&1 || { echo RUN_FAIL tp8sim_$pl; tail -30 gpurun_out/r5/a_tp8sim_$pl.log; exit 1; }
  summ gpurun_out/r5/a_tp8sim_$pl.log tp8sim_$pl
done
env OGKM_SHARDS_PLANNER=off OGKM_UNIT_MIN_MB=0 OMP_NUM_THREADS=4 timeout -k 10 200 python -u bench.py --gpus 2 --same-gpu --launch-timeout 60 --parallel shards --model small --batch 8 --context 64 --steps 3 --warmup 2 --no-aux --weights ans --kv-format bf16 --oversub 1.5 > gpurun_out/r5/a_shards_off.log 2>&1
rc=$?
echo "shards_off rc=$rc"
grep -c "ogkm-hang" gpurun_out/r5/a_shards_off.log
tail -5 gpurun_out/r5/a_shards_off.log
