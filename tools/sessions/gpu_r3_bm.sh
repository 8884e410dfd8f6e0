#!/bin/bash
ulimit -c 0
mkdir -p gpurun_out/r3
for cfg in "256 1024 2" "64 256 4" "16 64 8"; do
  set -- $cfg
  timeout -k 10 150 python tools/bench_managed.py --tensors 8 --mb $1 --arena-mb $2 --iters $3 --mode dispatch > gpurun_out/r3/bm_d$1.log 2>&1 || exit $?
  tail -1 gpurun_out/r3/bm_d$1.log
done
