#!/bin/bash
# Round 5 (ah): final build - the whole GPU suite, smoke(), the default bench,
# config 2, the transparent 70B.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/ah_gpu_suite.log 2>&1 || { echo SUITE_FAIL; tail -40 gpurun_out/r5/ah_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r5/ah_gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/ah_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r5/ah_smoke.log; exit 1; }
tail -1 gpurun_out/r5/ah_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r5/ah_bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r5/ah_bench.log; exit 1; }
grep '^{' gpurun_out/r5/ah_bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['steps'], d['warmup'])"
timeout -k 10 400 python -u bench.py --no-aux --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r5/ah_c2.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r5/ah_c2.log; exit 1; }
grep '^{' gpurun_out/r5/ah_c2.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'])"
OGKM_PACK=1 timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/ah_tm.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r5/ah_tm.log; exit 1; }
grep '^{' gpurun_out/r5/ah_tm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'])"
echo ALL_OK
