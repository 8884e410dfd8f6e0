#!/bin/bash
# Decode GEMM: row-tile-per-wave (wg) vs 4-row-tile waves at Llama-3-8B and 70B shapes (M = 64, raw bf16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_dgemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dgemm_tests.log 2>&1; rc=$?
tail -1 gpurun_out/dgemm_tests.log; grep -E "^(FAILED|E )" gpurun_out/dgemm_tests.log | head -4
for wg in 0; do for units in 1024 2048 4096; do
  OGKM_DGEMM_WG=$wg SHAPES=6144x4096,4096x4096,28672x4096,4096x14336 OGKM_DGEMM_UNITS=$units VARIANTS=raw:2,raw:4,raw:8 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/8b wg=$wg units=$units /" | cut -c1-200
done; done
for wg in 0; do
  OGKM_DGEMM_WG=$wg OGKM_DGEMM_UNITS=2048 VARIANTS=raw:4 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | sed "s/^/70b wg=$wg /" | cut -c1-220
done
