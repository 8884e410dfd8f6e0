#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_codec.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/codec_tests.log 2>&1; rc=$?
tail -1 gpurun_out/codec_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|E )" gpurun_out/codec_tests.log | head; exit 1; }
timeout -k 10 900 python -u bench.py --context 32768 --batch 8 --kv-format ans --kv-tiering --steps 3 --warmup 1 --no-aux > gpurun_out/longctx_ans.log 2>&1 || { echo LONGCTX_FAIL; tail -20 gpurun_out/longctx_ans.log; exit 1; }
grep '^{' gpurun_out/longctx_ans.log | cut -c1-700
