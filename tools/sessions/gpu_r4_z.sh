#!/bin/bash
# Round 4: planner off - capacity-ratio spread classes.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_b() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --planner off --steps 4 --warmup 3 --no-aux > gpurun_out/r4/z_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r4/z_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/z_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['ring_per_step'])"
}
run_b k097 X=1 && run_b k090 OGKM_SPREAD_KEEP=0.90 && run_b k100 OGKM_SPREAD_KEEP=1.0 && run_b k080 OGKM_SPREAD_KEEP=0.80 || exit 1
echo ALL_OK
