#!/bin/bash
# Final round check: full GPU suite + smoke + headline, then the long-context packed-KV line.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_verify.sh || exit 1
timeout -k 10 900 python -u bench.py --context 32768 --batch 8 --kv-format ans --kv-tiering --steps 3 --warmup 1 --no-aux > gpurun_out/longctx_ans.log 2>&1 || { echo LONGCTX_FAIL; tail -20 gpurun_out/longctx_ans.log; exit 1; }
grep '^{' gpurun_out/longctx_ans.log | cut -c1-700
