#!/bin/bash
# Round 5 (s): decode-attention A/B variants (OGKM_ATTN_VAR 0-3: TH4 / early V),
# numerics of each, graph-timed rates.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
for v in 0 1 2 3; do
  OGKM_ATTN_VAR=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused.py -k "attention and not kv_rate" > gpurun_out/r5/s_attn_tests_$v.log 2>&1 || { echo ATTN_TESTS_FAIL $v; tail -30 gpurun_out/r5/s_attn_tests_$v.log; exit 1; }
  echo "var $v tests: $(tail -1 gpurun_out/r5/s_attn_tests_$v.log)"
  OGKM_ATTN_VAR=$v timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/s_attn_$v.txt 2>&1 || { echo ATTN_FAIL $v; tail -20 gpurun_out/r5/s_attn_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r5/s_attn_$v.txt | sed "s/^/var $v /"
done
echo ALL_OK
