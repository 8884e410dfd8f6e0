#!/bin/bash
# Round 5 (q): UnitStream hold mode (config 2 planner off vs static), 70B headline, tp8 sim.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; s=a.get('stream_stats_per_step') or {}; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], {k: s.get(k) for k in ('held','hold_drops','use_ms','acquire_ms','prefetch_ms','demand','refused')})"; }
run_b() {
  local tag=$1; shift
  timeout -k 10 500 python -u bench.py --no-aux "$@" > gpurun_out/r5/q_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/q_$tag.log; return 1; }
  summ gpurun_out/r5/q_$tag.log $tag
}
run_b c2_off --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b c2_off_b --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static_b --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b 70b --steps 6 --warmup 4 && \
run_b tp8sim --simulate-tp 8 --steps 8 --warmup 3 || exit 1
echo ALL_OK
