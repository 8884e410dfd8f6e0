#!/bin/bash
# round 6 (l): SDMA engine diagnostics of the BF12 staged refill (old tree vs
# new), the segmented-copy GPU tests, then the transparent 70B with segmented
# packed host copies on vs off (same box).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
(cd old_tree && RT_LOG=info timeout -k 10 200 python -u diag_bf12_refill.py > ../gpurun_out/r6/l_old.log 2>&1); grep -E "SDMA|staged|fused" gpurun_out/r6/l_old.log
RT_LOG=info timeout -k 10 200 python -u tools/diag_bf12_refill.py > gpurun_out/r6/l_new.log 2>&1; grep -E "SDMA|staged|fused" gpurun_out/r6/l_new.log
timeout -k 10 300 python -u -m pytest tests/test_packing_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r6/l_pack_tests.log 2>&1; tail -2 gpurun_out/r6/l_pack_tests.log
summ() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['host_ms_per_step'], a['ring_per_step']); print(json.dumps(a['block_census'])); print(a['pack'])"; }
OGKM_TM_CENSUS=1 timeout -k 10 900 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/l_tm70b_seg.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r6/l_tm70b_seg.log; exit 1; }
summ gpurun_out/r6/l_tm70b_seg.log seg_on
RT_PACK_SEGMENTS=0 OGKM_TM_CENSUS=1 timeout -k 10 900 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/l_tm70b_noseg.log 2>&1 || { echo TM_FAIL2; tail -30 gpurun_out/r6/l_tm70b_noseg.log; exit 1; }
summ gpurun_out/r6/l_tm70b_noseg.log seg_off
echo ALL_OK
