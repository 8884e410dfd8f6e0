#!/bin/bash
# Round 5 (j): packed host copies on the GPU (runtime DECODE_ANS path) - GPU
# tests, transparent 8B / 70B with packing, config 2 release batching.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_managed_mode_gpu.py -k undeclared > gpurun_out/r5/j_tests.log 2>&1 || { echo TESTS_FAIL; tail -60 gpurun_out/r5/j_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r5/j_tests.log | tail -12
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('stream_stats_per_step'))"; }
run_b() {
  local tag=$1; shift
  timeout -k 10 500 python -u bench.py --no-aux "$@" > gpurun_out/r5/j_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/j_$tag.log; return 1; }
  summ gpurun_out/r5/j_$tag.log $tag
}
run_tm() {  # $1 = tag, $2 = model, $3 = OGKM_PACK
  OGKM_PACK=$3 timeout -k 10 1000 python -u bench.py --torch-managed --model $2 --oversub 2 --steps 3 --warmup 3 > gpurun_out/r5/j_tm_$1.log 2>&1 || { echo TM_FAIL $1; tail -30 gpurun_out/r5/j_tm_$1.log; return 1; }
  grep '^{' gpurun_out/r5/j_tm_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm_$1', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'], a.get('pack'))"
}
run_b c2_b1 --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
RT_UNIT_RELEASE_BATCH=4 run_b c2_b4 --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
RT_UNIT_RELEASE_BATCH=8 run_b c2_b8 --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_tm 8b_pack llama3-8b 1 && run_tm 70b_pack llama3-70b 1 || exit 1
echo ALL_OK
