#!/bin/bash
# Round 4: config 2 and the headline after the planner-off resident fallback.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 200 python bench.py --model llama3-8b --oversub 1 --steps 30 --warmup 5 --no-aux > gpurun_out/r4/c2fix.log 2>&1 || { echo C2_FAIL; tail -20 gpurun_out/r4/c2fix.log; exit 1; }
grep '^{' gpurun_out/r4/c2fix.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['config']['planner'])"
timeout -k 10 400 python -u bench.py > gpurun_out/r4/c2fix_headline.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r4/c2fix_headline.log; exit 1; }
grep '^{' gpurun_out/r4/c2fix_headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline', d['value'], d['ms_per_step'], d['config']['planner'], d['aux']['traffic_per_step_gb']['pcie_measured'])"
echo ALL_OK
