#!/bin/bash
# Round 5 (ae): the round-end checks the driver runs - the whole GPU suite,
# smoke(), the default bench.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/ae_gpu_suite.log 2>&1 || { echo SUITE_FAIL; tail -40 gpurun_out/r5/ae_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r5/ae_gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/ae_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r5/ae_smoke.log; exit 1; }
tail -1 gpurun_out/r5/ae_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r5/ae_bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r5/ae_bench.log; exit 1; }
grep '^{' gpurun_out/r5/ae_bench.log | tail -1 | cut -c1-400
timeout -k 10 700 python -u bench.py --no-aux --context 32768 --batch 8 --kv-tiering --steps 3 --warmup 2 > gpurun_out/r5/ae_longctx.log 2>&1 || { echo LC_FAIL; tail -30 gpurun_out/r5/ae_longctx.log; exit 1; }
grep '^{' gpurun_out/r5/ae_longctx.log | tail -1 | cut -c1-300
echo ALL_OK
