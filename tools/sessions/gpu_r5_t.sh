#!/bin/bash
# Round 5 (t): config 2 hold-mode diagnostics, attention variants, transparent
# 70B after the DMA pointer-lookup cache.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_packing_gpu.py > gpurun_out/r5/t_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r5/t_tests.log; exit 1; }
tail -1 gpurun_out/r5/t_tests.log
timeout -k 10 500 python -u bench.py --no-aux --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r5/t_c2_off.log 2>&1 || { echo RUN_FAIL; tail -30 gpurun_out/r5/t_c2_off.log; exit 1; }
grep '^{' gpurun_out/r5/t_c2_off.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2_off', d['value'], d['ms_per_step'], d['aux'].get('stream_stats_per_step'))"
for v in 0 1 2 3; do
  OGKM_ATTN_VAR=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused.py -k "attention and not kv_rate" > gpurun_out/r5/t_attn_tests_$v.log 2>&1 || { echo ATTN_TESTS_FAIL $v; tail -30 gpurun_out/r5/t_attn_tests_$v.log; exit 1; }
  echo "var $v tests: $(tail -1 gpurun_out/r5/t_attn_tests_$v.log)"
  OGKM_ATTN_VAR=$v timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/t_attn_$v.txt 2>&1 || { echo ATTN_FAIL $v; tail -20 gpurun_out/r5/t_attn_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r5/t_attn_$v.txt | sed "s/^/var $v /"
done
OGKM_PACK=1 timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/t_tm.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r5/t_tm.log; exit 1; }
grep '^{' gpurun_out/r5/t_tm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
echo ALL_OK
