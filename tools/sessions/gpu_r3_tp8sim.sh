#!/bin/bash
# TP code path (world > 1 branches: unfused epilogues, all-reduce, vocab-parallel
# argmax) on real kernels: the 70B tp8 rank-0 shard simulated on 1 GPU, with a
# one-rank RCCL group so every collective still runs.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
OGKM_DIST_FORCE=1 timeout -k 10 500 python -u bench.py --simulate-tp 8 --steps 8 --warmup 3 > gpurun_out/r3/tp8sim.log 2>&1 || { echo TP8_FAIL; tail -30 gpurun_out/r3/tp8sim.log; exit 1; }
grep '^{' gpurun_out/r3/tp8sim.log | cut -c1-400
echo ALL_OK
