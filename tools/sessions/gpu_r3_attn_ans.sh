#!/bin/bash
# Decode attention with / without the V preload (all shapes) and the HBM unpack
# kernels' throughput + bit-exactness after the deeper prefetch.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 200 python -u -m pytest tests/test_gpu_runtime.py -k "unpack_hbm or corrupt" tests/test_fused.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r3/attn_ans_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r3/attn_ans_tests.log; exit 1; }
grep -E "HBM unpack|passed|failed" gpurun_out/r3/attn_ans_tests.log
for v in 0 1; do OGKM_ATTN_VPRE=$v timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids; done
echo ALL_OK
