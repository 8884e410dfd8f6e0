#!/bin/bash
# Round 4: host profile of the planner-off 70B step; 70B stock-torch managed lookahead probe.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u tools/prof_host_step.py --model llama3-70b --simulate-tp 1 --planner off --steps 2 --warmup 3 > gpurun_out/r4/g_prof_off.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/r4/g_prof_off.log; exit 1; }
head -40 gpurun_out/r4/g_prof_off.log
for la in 0 2048; do
  OGKM_MANAGED_LOOKAHEAD_MB=$la timeout -k 10 900 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/g_tm70_$la.log 2>&1 || { echo TM70_FAIL; tail -30 gpurun_out/r4/g_tm70_$la.log; exit 1; }
  grep '^{' gpurun_out/r4/g_tm70_$la.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('la', $la, d['value'], d['ms_per_step'], {k: a[k] for k in ('htd_gb_per_step','dth_gb_per_step','link_gbps','evictions','faulted_ops','prefetches','trace_len','hinted_ops','trace_misses','ops','host_ms_per_step')})"
done
echo ALL_OK
