#!/bin/bash
# Kernel profile of the config-2 path (8B, HBM-resident, batch 64, ctx 1024).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run -- python bench.py --model llama3-8b --oversub 1.0 --steps 10 --warmup 3 --no-aux > gpurun_out/prof8b.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof8b.log; exit 1; }
grep '^{' gpurun_out/prof8b.log | cut -c1-200
f=$(find gpurun_out/prof8b -name "*kernel_stats.csv" | head -1); echo $f; head -25 "$f" | cut -c1-220
