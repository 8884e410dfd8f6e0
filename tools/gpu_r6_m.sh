#!/bin/bash
# round 6 (m): GPU tests of this round's paths, transparent 70B with segmented
# host copies, headline bench, attention split A/B, config 2 (arena allocator
# default) + its kernel profile (kernel trace only).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 400 python -u -m pytest tests/test_packing_gpu.py tests/test_gpu_runtime.py -q -s -k "packing or segment or packed or allocator or bf12" --timeout 120 --timeout-method thread > gpurun_out/r6/m_tests.log 2>&1; rc=$?
grep -E "refill 1 GiB|single-segment|passed|failed" gpurun_out/r6/m_tests.log | cut -c1-300
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/m_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r6/m_smoke.log; exit 1; }
grep -o "max_logit_err_vs_fp32': [0-9.]*" gpurun_out/r6/m_smoke.log
summ() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['host_ms_per_step'], a['ring_per_step']); print(json.dumps(a['block_census'])); print(a['pack'])"; }
OGKM_TM_CENSUS=1 timeout -k 10 900 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/m_tm70b_seg.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r6/m_tm70b_seg.log; exit 1; }
summ gpurun_out/r6/m_tm70b_seg.log seg_on
echo ALL_OK
