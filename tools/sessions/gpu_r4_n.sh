#!/bin/bash
# Round 4: DMA ring worker timing (fence waits / copies / idle) - static plan, planner off, stock-torch 70B.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
for mode in static off; do
  timeout -k 10 400 python -u bench.py --planner $mode --steps 4 --warmup 3 --no-aux > gpurun_out/r4/n_$mode.log 2>&1 || { echo RUN_FAIL $mode; tail -30 gpurun_out/r4/n_$mode.log; exit 1; }
  grep '^{' gpurun_out/r4/n_$mode.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['ring_per_step'])"
done
timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/n_tm70.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r4/n_tm70.log; exit 1; }
grep '^{' gpurun_out/r4/n_tm70.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm70', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
echo ALL_OK
