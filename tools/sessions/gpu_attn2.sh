#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1; rc=$?
tail -2 gpurun_out/attn_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E )" gpurun_out/attn_tests.log | head -20; exit 1; }
timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_attn.txt
timeout -k 10 300 python bench.py --model llama3-8b --oversub 1.0 --steps 10 --warmup 3 --no-aux > gpurun_out/b8.log 2>&1 && grep '^{' gpurun_out/b8.log | cut -c1-160
