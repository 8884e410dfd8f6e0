#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1; rc=$?
tail -1 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|E )" gpurun_out/attn_tests.log | head; exit 1; }
timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
