#!/bin/bash
# Decode-GEMM sweep with MALL-cold weights (bench_dgemm COLD=1): k_dgemm_pipe vs
# the LDS ring at several wave counts, 8B and 70B decode shapes.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
S8="6144x4096,4096x4096,14336x4096,4096x14336,128256x4096"
for U in 512 1024 1536; do
  V="pipe:30,pipe:40,pipe:50,pipe:70"
  [ $U = 512 ] && V="pipe:4,$V"
  SHAPES=$S8 VARIANTS=$V OGKM_DGEMM_LRING_UNITS=$U timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/cold8b_$U.jsonl 2>&1 || { echo B8_FAIL; tail -20 gpurun_out/r3/cold8b_$U.jsonl; exit 1; }
  VARIANTS=$V OGKM_DGEMM_LRING_UNITS=$U timeout -k 10 300 python -u tools/bench_dgemm.py > gpurun_out/r3/cold70b_$U.jsonl 2>&1 || { echo B70_FAIL; tail -20 gpurun_out/r3/cold70b_$U.jsonl; exit 1; }
  echo "units $U"; grep '^{' gpurun_out/r3/cold8b_$U.jsonl | cut -c1-360; grep '^{' gpurun_out/r3/cold70b_$U.jsonl | cut -c1-330
done
echo ALL_OK
