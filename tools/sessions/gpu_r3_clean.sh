#!/bin/bash
# Clean-first eviction: stock-torch 8B managed mode A/B, headline 70B and
# planner-off (runtime-decided residency) unaffected-check, managed GPU tests.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
for C in 1 0; do
  RT_EVICT_CLEAN_FIRST=$C timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r3/cl_tm$C.log 2>&1 || { echo TM_FAIL $C; tail -30 gpurun_out/r3/cl_tm$C.log; exit 1; }
  echo "clean_first $C $(grep '^{' gpurun_out/r3/cl_tm$C.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); a=d["aux"]; print(d["value"], d["ms_per_step"], a["htd_gb_per_step"], a["dth_gb_per_step"], a["link_gbps"], a["tlb_flushes"])')"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_managed_mode.py tests/test_allocator.py > gpurun_out/r3/cl_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r3/cl_tests.log; exit 1; }
tail -1 gpurun_out/r3/cl_tests.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3/cl_h70.log 2>&1 || { echo H70_FAIL; tail -30 gpurun_out/r3/cl_h70.log; exit 1; }
echo "70b $(grep '^{' gpurun_out/r3/cl_h70.log | cut -c1-160)"
timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --planner off > gpurun_out/r3/cl_poff.log 2>&1 || { echo POFF_FAIL; tail -30 gpurun_out/r3/cl_poff.log; exit 1; }
echo "planner-off $(grep '^{' gpurun_out/r3/cl_poff.log | cut -c1-160)"
echo ALL_OK
