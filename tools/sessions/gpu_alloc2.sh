#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -k "allocator or managed" -x -q --timeout 120 --timeout-method thread > gpurun_out/alloc_tests.log 2>&1; rc=$?
tail -1 gpurun_out/alloc_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|E )" gpurun_out/alloc_tests.log | head; exit 1; }
timeout -k 10 300 python bench.py --model llama3-8b --oversub 1.0 --allocator --steps 10 --warmup 3 --no-aux > gpurun_out/b8a.log 2>&1 && grep '^{' gpurun_out/b8a.log | cut -c1-160
