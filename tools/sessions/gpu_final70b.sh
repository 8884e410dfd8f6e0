#!/bin/bash
# Default 70B bench (ans weights + ans KV, SDMA ring), the bf11-KV variant, and a kernel-trace profile
# of the default. Each step time-limited; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/f_default.log 2>&1 || { echo DEF_FAIL; tail -20 gpurun_out/f_default.log; exit 1; }
grep '^{' gpurun_out/f_default.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-aux --kv-format bf11 > gpurun_out/f_kvbf11.log 2>&1 || { echo KV_FAIL; tail -20 gpurun_out/f_kvbf11.log; exit 1; }
grep '^{' gpurun_out/f_kvbf11.log | cut -c1-160
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o k -- python $R/bench.py --steps 3 --warmup 1 --no-aux > gpurun_out/prof_final.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_final.log; exit 1; }
python tools/trace_gaps.py gpurun_out/prof_final --last-ms 2500 > gpurun_out/trace_gaps_final.txt 2>&1; head -3 gpurun_out/trace_gaps_final.txt
