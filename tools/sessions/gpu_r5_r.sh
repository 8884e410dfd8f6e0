#!/bin/bash
# Round 5 (r): why UnitStream hold mode does not engage in config 2 (diagnostic counters).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 500 python -u bench.py --no-aux --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r5/r_c2_off.log 2>&1 || { echo RUN_FAIL; tail -30 gpurun_out/r5/r_c2_off.log; exit 1; }
grep '^{' gpurun_out/r5/r_c2_off.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['aux'].get('stream_stats_per_step'))"
echo ALL_OK
