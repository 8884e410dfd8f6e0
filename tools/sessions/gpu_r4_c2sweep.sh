#!/bin/bash
# Round 4: config-2 decode GEMM launch-shape sweep (LDS-ring waves / depth).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_c2() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --model llama3-8b --oversub 1 --steps 30 --warmup 5 --no-aux > gpurun_out/r4/c2s_$tag.log 2>&1 || { echo C2_FAIL $tag; tail -20 gpurun_out/r4/c2s_$tag.log; return 1; }
  echo "$tag $(grep '^{' gpurun_out/r4/c2s_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
run_c2 base X=1 && run_c2 u384 OGKM_DGEMM_LRING_UNITS=384 && run_c2 u768 OGKM_DGEMM_LRING_UNITS=768 && run_c2 d60 OGKM_DGEMM_LRING_DEPTH=60 && run_c2 d70 OGKM_DGEMM_LRING_DEPTH=70 && run_c2 d40 OGKM_DGEMM_LRING_DEPTH=40 || exit 1
echo ALL_OK
