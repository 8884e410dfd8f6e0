#!/bin/bash
# Attention kernel: fp32-reference tests, then the 8B config-2 profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1; rc=$?
tail -3 gpurun_out/attn_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E )" gpurun_out/attn_tests.log | head -20; exit 1; }
rm -rf gpurun_out/prof8b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run -- python bench.py --model llama3-8b --oversub 1.0 --steps 10 --warmup 3 --no-aux > gpurun_out/prof8b.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof8b.log; exit 1; }
grep '^{' gpurun_out/prof8b.log | cut -c1-200
