#!/bin/bash
# Decode GEMM: LDS-shared activations (OGKM_DGEMM_LDS=1) vs the 4-row-tile kernel; numerics first.
set -o pipefail
mkdir -p gpurun_out
OGKM_DGEMM_LDS=1 timeout -k 10 200 python -u -m pytest tests/test_dgemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dgemm_lds_tests.log 2>&1; rc=$?
tail -1 gpurun_out/dgemm_lds_tests.log; grep -E "^(FAILED|E )" gpurun_out/dgemm_lds_tests.log | head -4
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for units in 768 1536 3072; do
  OGKM_DGEMM_LDS=1 SHAPES=6144x4096,4096x4096,28672x4096,4096x14336 OGKM_DGEMM_UNITS=$units VARIANTS=raw:2,raw:4,raw:8 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/8b lds units=$units /" | cut -c1-130
  OGKM_DGEMM_LDS=1 OGKM_DGEMM_UNITS=$units VARIANTS=raw:4,raw:8 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/70b lds units=$units /" | cut -c1-130
done
SHAPES=6144x4096,4096x4096,28672x4096,4096x14336 VARIANTS=raw:2 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/8b base /" | cut -c1-130
VARIANTS=raw:2 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/70b base /" | cut -c1-130
