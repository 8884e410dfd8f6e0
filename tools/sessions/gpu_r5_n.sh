#!/bin/bash
# Round 5 (n): bisect the managed-mode bit mismatch (deferred decode publish /
# packing), attention all-in-flight variant numerics + rate.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
T="tests/test_managed_mode_gpu.py::test_stock_transformer_oversubscribed_bitwise"
for v in "RT_RING_DEFER_DECODES=1" "RT_RING_DEFER_DECODES=0" "RT_PACK_HOST_COPIES=0"; do
  env $v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "$T" > gpurun_out/r5/n_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r5/n_$v.log)"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused.py -k attention > gpurun_out/r5/n_attn_tests.log 2>&1 || { echo ATTN_TESTS_FAIL; tail -30 gpurun_out/r5/n_attn_tests.log; exit 1; }
tail -1 gpurun_out/r5/n_attn_tests.log
timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/n_attn.txt 2>&1 && OGKM_ATTN_ALL=0 timeout -k 10 180 python -u tools/bench_attn.py >> gpurun_out/r5/n_attn.txt 2>&1 && OGKM_ATTN_ALL=1 timeout -k 10 180 python -u tools/bench_attn.py >> gpurun_out/r5/n_attn.txt 2>&1 || { echo ATTN_FAIL; tail -20 gpurun_out/r5/n_attn.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/n_attn.txt
echo ALL_OK
