#!/bin/bash
# Round 4: planner off - a deep, missing-bytes prefetch window to carry the link across Belady's resident run.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_b() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --planner off --steps 4 --warmup 3 --no-aux > gpurun_out/r4/s_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r4/s_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/s_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['ring_per_step'], d['aux']['stream_stats_per_step'])"
}
run_b w2g OGKM_WINDOW_MISSING=1 OGKM_WINDOW_MB=2048 OGKM_MAX_AHEAD=64 && run_b w4g OGKM_WINDOW_MISSING=1 OGKM_WINDOW_MB=4096 OGKM_MAX_AHEAD=64 && run_b w8g OGKM_WINDOW_MISSING=1 OGKM_WINDOW_MB=8192 OGKM_MAX_AHEAD=128 || exit 1
echo ALL_OK
