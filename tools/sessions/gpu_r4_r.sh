#!/bin/bash
# Round 4: planner-off late uses (bytes not placed in HBM when a unit is used), next-use vs workingset.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_b() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --planner off --steps 4 --warmup 3 --no-aux --verbose > gpurun_out/r4/r_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r4/r_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/r_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['ring_per_step'], d['aux']['stream_stats_per_step'])"
  grep "H2D bytes/step around" gpurun_out/r4/r_$tag.log | cut -c1-600
}
run_b nu X=1 && run_b nonu OGKM_NEXT_USE=0 || exit 1

timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/r_tm70.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r4/r_tm70.log; exit 1; }
grep '^{' gpurun_out/r4/r_tm70.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm70', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
echo ALL_OK
