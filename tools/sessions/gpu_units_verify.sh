#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for units in 512 768 1024 2048; do
  SHAPES=6144x4096,4096x4096,28672x4096,4096x14336 OGKM_DGEMM_UNITS=$units VARIANTS=raw:2,raw:4 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/8b units=$units /" | cut -c1-120
  OGKM_DGEMM_UNITS=$units VARIANTS=raw:2,raw:4 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/70b units=$units /" | cut -c1-120
done
bash tools/gpu_verify.sh
