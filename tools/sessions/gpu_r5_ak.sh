#!/bin/bash
# Round 5 (ak): one-round split combine - numerics, attention rates, the combine's
# time at the tp8 shape, config 2.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_fused.py tests/test_model_gpu.py > gpurun_out/r5/ak_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r5/ak_tests.log; exit 1; }
tail -1 gpurun_out/r5/ak_tests.log
grep "TB/s of KV" gpurun_out/r5/ak_tests.log
timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/ak_attn.txt 2>&1 || { echo ATTN_FAIL; tail -20 gpurun_out/r5/ak_attn.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/ak_attn.txt
timeout -k 10 400 python -u bench.py --no-aux --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r5/ak_c2.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r5/ak_c2.log; exit 1; }
grep '^{' gpurun_out/r5/ak_c2.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'])"
cd /tmp && SHAPE=70b-tp8 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/ak_prof_tp8 -o attn -- python3 $R/tools/bench_attn.py > $R/gpurun_out/r5/ak_prof_tp8.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/r5/ak_prof_tp8.log; exit 1; }
cd $R && python3 tools/rocpd_summary.py gpurun_out/r5/ak_prof_tp8/attn_results.db 4 --last-ms 1
echo ALL_OK
