#!/bin/bash
# Round 4: planner-off 70B - residency-aware prefetch window and host run-ahead variants.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_off() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --planner off --steps 6 --warmup 3 --no-aux --verbose > gpurun_out/r4/i_off_$tag.log 2>&1 || { echo OFF_FAIL $tag; tail -30 gpurun_out/r4/i_off_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/i_off_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['evictions'])"
}
run_off missing1 OGKM_WINDOW_MISSING=1 && run_off missing0 OGKM_WINDOW_MISSING=0 && run_off ahead8 OGKM_WINDOW_MISSING=1 OGKM_MAX_AHEAD=8 && run_off win768 OGKM_WINDOW_MISSING=1 OGKM_WINDOW_MB=768 || exit 1
echo ALL_OK
