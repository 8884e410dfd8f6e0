#!/bin/bash
# Round 5 (b): headline after the issued-before-GPU-wait ordering, 405B tp8-shard
# simulation (3 tiers) planner off vs static, then the 2-rank peer-shard run
# under planner off (round-4 hang) and the tp2 GPU test with it.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['config']['planner'], d['aux']['traffic_per_step_gb'], d['aux'].get('stream_stats_per_step'), d['aux'].get('ring_per_step'))"; }
timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --no-aux > gpurun_out/r5/b_70b.log 2>&1 || { echo RUN_FAIL 70b; tail -30 gpurun_out/r5/b_70b.log; exit 1; }
summ gpurun_out/r5/b_70b.log 70b_off
for pl in off static; do
  timeout -k 10 500 python -u bench.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --planner $pl --steps 6 --warmup 3 --no-aux > gpurun_out/r5/b_405_$pl.log 2>&1 || { echo RUN_FAIL 405_$pl; tail -30 gpurun_out/r5/b_405_$pl.log; exit 1; }
  summ gpurun_out/r5/b_405_$pl.log 405tp8sim_$pl
done
env OGKM_SHARDS_PLANNER=off OGKM_UNIT_MIN_MB=0 OMP_NUM_THREADS=4 timeout -k 10 200 python -u bench.py --gpus 2 --same-gpu --launch-timeout 60 --parallel shards --model small --batch 8 --context 64 --steps 3 --warmup 2 --no-aux --weights ans --kv-format bf16 --oversub 1.5 > gpurun_out/r5/b_shards_off.log 2>&1
rc=$?
echo "shards_off rc=$rc"
grep '^{' gpurun_out/r5/b_shards_off.log | head -c 300; echo
[ $rc -eq 0 ] || { grep "ogkm-dump\]   ring cpu\|engine\|lease " gpurun_out/r5/b_shards_off.log | head; exit 1; }
env OGKM_SHARDS_PLANNER=off timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tp2.py > gpurun_out/r5/b_tp2.log 2>&1; rc=$?
tail -5 gpurun_out/r5/b_tp2.log
exit $rc
