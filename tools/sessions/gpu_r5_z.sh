#!/bin/bash
# Round 5 (z): 1024-thread RMSNorm for decode batches - numerics, config 2 A/B.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused.py tests/test_model_gpu.py > gpurun_out/r5/z_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r5/z_tests.log; exit 1; }
tail -1 gpurun_out/r5/z_tests.log
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['config']['planner'])"; }
run_b() {
  local tag=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --no-aux --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r5/z_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/z_$tag.log; return 1; }
  summ gpurun_out/r5/z_$tag.log $tag
}
run_b norm1k OGKM_NORM_1K=1 && run_b norm256 OGKM_NORM_1K=0 && run_b norm1k_b OGKM_NORM_1K=1 && run_b norm256_b OGKM_NORM_1K=0 || exit 1
timeout -k 10 700 python -u bench.py --no-aux --context 32768 --batch 8 --kv-tiering --steps 3 --warmup 2 > gpurun_out/r5/z_longctx.log 2>&1 || { echo LONGCTX_FAIL; tail -30 gpurun_out/r5/z_longctx.log; exit 1; }
summ gpurun_out/r5/z_longctx.log longctx
echo ALL_OK
