#!/bin/bash
# Round 5 (an): the exact final tree - GPU suite + smoke().
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/an_gpu_suite.log 2>&1 || { echo SUITE_FAIL; tail -40 gpurun_out/r5/an_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r5/an_gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/an_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r5/an_smoke.log; exit 1; }
tail -1 gpurun_out/r5/an_smoke.log
echo ALL_OK
