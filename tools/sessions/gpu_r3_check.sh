#!/bin/bash
# Round-3 check: GPU suite, smoke, 70B headline (with the HBM<->host/CXL probe),
# config 2 (8B HBM-resident), the stock-torch managed-mode bench. Each step
# time-limited; stop at the first failure.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
bash tools/gpu_verify.sh || exit 1
timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 10 --warmup 3 --no-aux > gpurun_out/r3/config2.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/config2.log; exit 1; }
grep '^{' gpurun_out/r3/config2.log | cut -c1-300
timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r3/tm8b.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r3/tm8b.log; exit 1; }
grep '^{' gpurun_out/r3/tm8b.log | cut -c1-1500
echo ALL_OK
