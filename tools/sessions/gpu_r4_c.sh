#!/bin/bash
# Round 4: planner-off floor-fallback A/B, stock-torch managed host profile.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u tools/prof_torch_managed.py --steps 2 > gpurun_out/r4/c_prof_tm.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/r4/c_prof_tm.log; exit 1; }
head -45 gpurun_out/r4/c_prof_tm.log
for v in "OGKM_FLOOR_FALLBACK=plain" "OGKM_NEXT_USE=0"; do
  env $v timeout -k 10 600 python -u bench.py --planner off --steps 8 --warmup 3 --no-aux > gpurun_out/r4/c_off.log 2>&1 || { echo OFF_FAIL; tail -30 gpurun_out/r4/c_off.log; exit 1; }
  grep '^{' gpurun_out/r4/c_off.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['evictions'])"
done
echo ALL_OK
