#!/bin/bash
# GPU tests, smoke, default 70B bench, then the rANS-weights variant. Each step time-limited; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_verify.sh || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-aux --weights ans ${ANS_ARGS} > gpurun_out/bench70b_ans.log 2>&1 || { echo ANS_FAIL; tail -30 gpurun_out/bench70b_ans.log; exit 1; }
grep '^{' gpurun_out/bench70b_ans.log
