#!/bin/bash
# Stock-torch 8B managed mode (2x): prefetch-window sweep after the flush elision.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
for LA in 512 1024 2048 256; do
  OGKM_MANAGED_LOOKAHEAD_MB=$LA timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r3/tm_la$LA.log 2>&1 || { echo TM_FAIL $LA; tail -30 gpurun_out/r3/tm_la$LA.log; exit 1; }
  echo "la $LA $(grep '^{' gpurun_out/r3/tm_la$LA.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); a=d["aux"]; print(d["value"], d["ms_per_step"], a["htd_gb_per_step"], a["dth_gb_per_step"], a["link_gbps"], a["tlb_flushes"])')"
done
echo ALL_OK
