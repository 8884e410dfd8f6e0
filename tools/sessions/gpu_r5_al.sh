#!/bin/bash
# Round 5 (al): the final tree - whole GPU suite, smoke(), the default bench.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/al_gpu_suite.log 2>&1 || { echo SUITE_FAIL; tail -40 gpurun_out/r5/al_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r5/al_gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/al_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r5/al_smoke.log; exit 1; }
tail -1 gpurun_out/r5/al_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r5/al_bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r5/al_bench.log; exit 1; }
grep '^{' gpurun_out/r5/al_bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['steps'], d['warmup'])"
echo ALL_OK
