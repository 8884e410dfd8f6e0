#!/bin/bash
# Decode GEMM sweep (graph-timed): split-K kernels (old / pipelined, unit targets),
# fused; then the dgemm GPU numerics tests and the CXL path probe (preferred engines).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_dgemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/dgemm_tests.log 2>&1 || { echo DG_TESTS_FAIL; tail -30 gpurun_out/r3/dgemm_tests.log; exit 1; }
tail -2 gpurun_out/r3/dgemm_tests.log
S8="6144x4096,4096x4096,28672x4096,4096x14336"
run() {  # tag env...
  local tag=$1; shift
  env "$@" SHAPES=$S8 VARIANTS="raw:2" timeout -k 10 120 python -u tools/bench_dgemm.py > gpurun_out/r3/sw_8b_$tag.jsonl 2>&1 || return 1
  env "$@" VARIANTS="raw:2" timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/sw_70b_$tag.jsonl 2>&1 || return 1
  echo "$tag 8b $(grep '^{' gpurun_out/r3/sw_8b_$tag.jsonl | cut -c1-250)"
  echo "$tag 70b $(grep '^{' gpurun_out/r3/sw_70b_$tag.jsonl | cut -c1-250)"
}
run old OGKM_DGEMM_PIPE=0 || exit 1
run oldnolds OGKM_DGEMM_PIPE=0 OGKM_DGEMM_LDS=0 || exit 1
for u in 768 1024 1536 2048; do run pipe$u OGKM_DGEMM_PIPE=1 OGKM_DGEMM_LDS=0 OGKM_DGEMM_UNITS_PIPE=$u || exit 1; done
timeout -k 10 180 ./tools/bin/probe_cxl_paths 1024 > gpurun_out/r3/cxl_paths2.jsonl 2> gpurun_out/r3/cxl_paths2.err || { echo PROBE_FAIL; exit 1; }
head -2 gpurun_out/r3/cxl_paths2.jsonl
echo ALL_OK
