#!/bin/bash
# Round 4, first GPU call: the new 2-rank test, the GPU suite, and the stock-torch managed 8B baseline.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_tp2.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4/a_tp2.log 2>&1 || { echo TP2_FAIL; tail -60 gpurun_out/r4/a_tp2.log; exit 1; }
tail -3 gpurun_out/r4/a_tp2.log
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4/a_gpu.log 2>&1 || { echo GPU_FAIL; tail -60 gpurun_out/r4/a_gpu.log; exit 1; }
tail -3 gpurun_out/r4/a_gpu.log
timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r4/a_tm.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r4/a_tm.log; exit 1; }
grep '^{' gpurun_out/r4/a_tm.log
echo ALL_OK
