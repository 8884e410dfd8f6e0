#!/bin/bash
# Split-K decode GEMMs with one-wave workgroups (every CU busy) vs 4-wave ones.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
S8="6144x4096,4096x4096,28672x4096,4096x14336"
run() {  # tag variants env...
  local tag=$1 v=$2; shift 2
  env "$@" SHAPES=$S8 VARIANTS="$v" timeout -k 10 120 python -u tools/bench_dgemm.py > gpurun_out/r3/sw3_8b_$tag.jsonl 2>&1 || return 1
  env "$@" VARIANTS="$v" timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/sw3_70b_$tag.jsonl 2>&1 || return 1
  echo "$tag 8b $(grep '^{' gpurun_out/r3/sw3_8b_$tag.jsonl | cut -c1-250)"
  echo "$tag 70b $(grep '^{' gpurun_out/r3/sw3_70b_$tag.jsonl | cut -c1-250)"
}
for u in 512 768 1024 1536; do run split${u}w1 "raw:2" OGKM_DGEMM_UNITS=$u OGKM_DGEMM_WG=1 || exit 1; done
for u in 768 1024 1536; do run pipe${u}w1 "pipe:2" OGKM_DGEMM_UNITS_PIPE=$u OGKM_DGEMM_WG=1 || exit 1; done
run bf11w1 "bf11:2" OGKM_DGEMM_WG=1 || exit 1
run bf11w4 "bf11:2" OGKM_DGEMM_WG=4 || exit 1
echo ALL_OK
