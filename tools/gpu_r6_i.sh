#!/bin/bash
# round 6 (i): BF12 staged refill A/B (old ring vs new ring), then the
# transparent 70B (stock torch.nn under ogkm.managed(), 2x) with segmented
# packed host copies + block census.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
( cd old_tree && timeout -k 10 200 python -u -m pytest tests/test_gpu_runtime.py -q -s -k "bf12_decode_bandwidth" --timeout 120 --timeout-method thread -p no:cacheprovider > ../gpurun_out/r6/i_oldring.log 2>&1; grep -E "refill" ../gpurun_out/r6/i_oldring.log )
timeout -k 10 200 python -u -m pytest tests/test_gpu_runtime.py -q -s -k "bf12_decode_bandwidth" --timeout 120 --timeout-method thread > gpurun_out/r6/i_new.log 2>&1; grep -E "refill" gpurun_out/r6/i_new.log
OGKM_TM_CENSUS=1 timeout -k 10 900 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/i_tm70b_seg.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r6/i_tm70b_seg.log; exit 1; }
grep '^{' gpurun_out/r6/i_tm70b_seg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm seg', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['host_ms_per_step'], a['ring_per_step']); print(json.dumps(a['block_census'])); print(a['pack'])"
echo ALL_OK
