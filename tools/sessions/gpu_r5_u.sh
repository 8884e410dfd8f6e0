#!/bin/bash
# Round 5 (u): null-stream UnitStream (hold mode on the model's stream), early-V
# attention default, config 2 off vs static, 70B headline, tp8 attention trace.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; s=a.get('stream_stats_per_step') or {}; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], {k: s.get(k) for k in ('held','hold_drops','quiet_passes','loud_streaming','loud_evictions','use_ms','acquire_ms','wait_ms','prefetch_ms','demand','refused')})"; }
run_b() {
  local tag=$1; shift
  timeout -k 10 700 python -u bench.py --no-aux "$@" > gpurun_out/r5/u_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/u_$tag.log; return 1; }
  summ gpurun_out/r5/u_$tag.log $tag
}
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_fused.py tests/test_unit_stream.py tests/test_model_gpu.py > gpurun_out/r5/u_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r5/u_tests.log; exit 1; }
tail -1 gpurun_out/r5/u_tests.log
grep "TB/s of KV" gpurun_out/r5/u_tests.log
run_b c2_off --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b 70b --steps 6 --warmup 4 || exit 1
cd /tmp && SHAPE=70b-tp8 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5/u_prof_tp8 -o attn -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py > $GRAFT_REPO_ROOT/gpurun_out/r5/u_prof_tp8.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r5/u_prof_tp8.log; exit 1; }
cd $GRAFT_REPO_ROOT
grep -v amdgpu.ids gpurun_out/r5/u_prof_tp8.log | tail -3
find gpurun_out/r5/u_prof_tp8 -name "*kernel_stats.csv" -exec cat {} \;
echo ALL_OK
