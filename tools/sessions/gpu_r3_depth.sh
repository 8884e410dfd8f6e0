#!/bin/bash
# Decode-GEMM pipeline depth: numerics of the deep / LDS-ring variants, then a
# sweep at Llama-3 8B and 70B decode shapes (M = 64, graph-timed incl. reduce).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dgemm.py -k "depths or numerics" > gpurun_out/r3/depth_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r3/depth_tests.log; exit 1; }
tail -2 gpurun_out/r3/depth_tests.log
S8="6144x4096,4096x4096,28672x4096,4096x14336"
V="pipe:4,pipe:30,pipe:40,pipe:42,pipe:50,pipe:70"
for U in 512 768 1536; do
  SHAPES=$S8 VARIANTS=$V OGKM_DGEMM_UNITS_PIPE=$U OGKM_DGEMM_UNITS_PIPE_LARGE=$U timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/depth8b_$U.jsonl 2>&1 || { echo B8_FAIL; tail -20 gpurun_out/r3/depth8b_$U.jsonl; exit 1; }
  VARIANTS=$V OGKM_DGEMM_UNITS_PIPE=$U OGKM_DGEMM_UNITS_PIPE_LARGE=$U timeout -k 10 300 python -u tools/bench_dgemm.py > gpurun_out/r3/depth70b_$U.jsonl 2>&1 || { echo B70_FAIL; tail -20 gpurun_out/r3/depth70b_$U.jsonl; exit 1; }
  echo "units $U"; grep '^{' gpurun_out/r3/depth8b_$U.jsonl | cut -c1-330; grep '^{' gpurun_out/r3/depth70b_$U.jsonl | cut -c1-330
done
echo ALL_OK
