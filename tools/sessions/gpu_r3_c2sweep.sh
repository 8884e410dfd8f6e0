#!/bin/bash
# Config 2 sweep of the LDS-ring GEMM plan (waves, ring depth, max K steps).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
run() {
  env "$@" timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/c2sw.log 2>&1 || { echo C2_FAIL "$@"; tail -30 gpurun_out/r3/c2sw.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/r3/c2sw.log | cut -c90-150)"
}
run OGKM_DGEMM_LRING_UNITS=512
run OGKM_DGEMM_LRING_UNITS=384
run OGKM_DGEMM_LRING_UNITS=640
run OGKM_DGEMM_LRING_UNITS=768
run OGKM_DGEMM_LRING_DEPTH=40
run OGKM_DGEMM_LRING_DEPTH=60
run OGKM_DGEMM_LRING_DEPTH=70 OGKM_DGEMM_LRING_UNITS=384
run OGKM_DGEMM_LRING_MAX_STEPS=0
run OGKM_DGEMM_LRING_UNITS=512
echo ALL_OK
