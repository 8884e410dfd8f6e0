#!/bin/bash
# Host-side cost of a tp8-shard decode step (cProfile) + fused-op GPU tests.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 200 python -u -m pytest tests/test_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/fused_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r3/fused_tests.log; exit 1; }
tail -1 gpurun_out/r3/fused_tests.log
timeout -k 10 400 python -u tools/prof_host_step.py --model llama3-70b --simulate-tp 8 > gpurun_out/r3/host_tp8.txt 2>&1 || { echo HOST_FAIL; tail -30 gpurun_out/r3/host_tp8.txt; exit 1; }
head -45 gpurun_out/r3/host_tp8.txt
echo ALL_OK
