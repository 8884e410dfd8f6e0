#!/bin/bash
# Round 4: planner-off streaming diagnostics (prefetches, floor refusals, demand uses, host waits).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_b() {  # $1 = tag, $2 = planner, rest = env
  local tag=$1 pl=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --planner $pl --steps 4 --warmup 3 --no-aux > gpurun_out/r4/p_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r4/p_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/p_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['ring_per_step'], d['aux']['stream_stats_per_step'])"
}
run_b static static X=1 && run_b off off X=1 && run_b off_plain off OGKM_FLOOR_FALLBACK=plain && run_b off_nonu off OGKM_NEXT_USE=0 || exit 1
echo ALL_OK
