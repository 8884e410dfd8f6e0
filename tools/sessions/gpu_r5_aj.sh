#!/bin/bash
# Round 5 (aj): decode attention variant 4 (16 V loads per round) vs the default.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
OGKM_ATTN_VAR=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused.py -k "attention and not kv_rate" > gpurun_out/r5/aj_attn_tests.log 2>&1 || { echo ATTN_TESTS_FAIL; tail -30 gpurun_out/r5/aj_attn_tests.log; exit 1; }
echo "var 4 tests: $(tail -1 gpurun_out/r5/aj_attn_tests.log)"
for r in a b; do
for v in 2 4; do
  OGKM_ATTN_VAR=$v timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/aj_attn_${v}_$r.txt 2>&1 || { echo ATTN_FAIL $v; tail -20 gpurun_out/r5/aj_attn_${v}_$r.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r5/aj_attn_${v}_$r.txt | sed "s/^/var $v $r /"
done
done
echo ALL_OK
