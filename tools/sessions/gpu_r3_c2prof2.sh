#!/bin/bash
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_c2d -o run -- python bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/prof_c2d.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/prof_c2d.log; exit 1; }
grep '^{' gpurun_out/r3/prof_c2d.log | cut -c1-200
echo ALL_OK
