#!/bin/bash
# Round 4: GPU suite on the new transparent mode (page-granular holds, next-use
# eviction, remote fallback, OOM error), then the stock-torch managed 8B and a
# lookahead sweep.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_managed_mode_gpu.py tests/test_gpu_tp2.py -x -v --timeout 240 --timeout-method thread -m gpu > gpurun_out/r4/b_new.log 2>&1 || { echo NEW_FAIL; tail -80 gpurun_out/r4/b_new.log; exit 1; }
tail -3 gpurun_out/r4/b_new.log
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4/b_gpu.log 2>&1 || { echo GPU_FAIL; tail -60 gpurun_out/r4/b_gpu.log; exit 1; }
tail -3 gpurun_out/r4/b_gpu.log
for sp in 256 1064; do
  SPLIT=$sp timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/r4/b_attn_$sp.log 2>&1 || { echo ATTN_FAIL; tail -20 gpurun_out/r4/b_attn_$sp.log; exit 1; }
  cat gpurun_out/r4/b_attn_$sp.log
done
for la in -1 256 2048; do
  OGKM_MANAGED_LOOKAHEAD_MB=$la timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r4/b_tm_$la.log 2>&1 || { echo TM_FAIL $la; tail -30 gpurun_out/r4/b_tm_$la.log; exit 1; }
  grep '^{' gpurun_out/r4/b_tm_$la.log | cut -c1-120
  grep '^{' gpurun_out/r4/b_tm_$la.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('la', $la, d['value'], d['aux'])"
done
timeout -k 10 600 python -u bench.py --planner off --steps 10 --warmup 3 > gpurun_out/r4/b_off.log 2>&1 || { echo OFF_FAIL; tail -30 gpurun_out/r4/b_off.log; exit 1; }
grep '^{' gpurun_out/r4/b_off.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('planner_off', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb'], d['aux']['evictions'])"
echo ALL_OK
