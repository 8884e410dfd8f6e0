#!/bin/bash
# Repeat of the managed 8B and config 2 runs on another box (box variance check).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r3/f2_tm.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r3/f2_tm.log; exit 1; }
grep '^{' gpurun_out/r3/f2_tm.log | cut -c1-170
timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/f2_c2.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/f2_c2.log; exit 1; }
grep '^{' gpurun_out/r3/f2_c2.log | cut -c1-170
echo ALL_OK
