#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_verify.sh || exit 1
timeout -k 10 300 python bench.py --model llama3-8b --oversub 1.0 --steps 10 --warmup 3 --no-aux > gpurun_out/b8.log 2>&1 && grep '^{' gpurun_out/b8.log | cut -c1-160
