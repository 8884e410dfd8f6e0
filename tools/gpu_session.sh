#!/bin/bash
# One GPU session: smoke, 8B + 70B benches, and a rocprofv3 kernel-trace of the 8B decode.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 --verbose > gpurun_out/bench8b.log 2>&1 || { echo B8_FAIL; tail -30 gpurun_out/bench8b.log; exit 1; }
tail -1 gpurun_out/bench8b.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof8b -o k -- python $R/bench.py --model llama3-8b --steps 3 --warmup 1 --no-aux > gpurun_out/prof8b.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof8b.log; exit 1; }
timeout -k 10 700 python bench.py --steps 4 --warmup 2 --verbose > gpurun_out/bench70b.log 2>&1 || { echo B70_FAIL; tail -30 gpurun_out/bench70b.log; exit 1; }
tail -1 gpurun_out/bench70b.log
