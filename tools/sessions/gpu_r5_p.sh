#!/bin/bash
# Round 5 (p): deferred decodes vs pipelined copies fixed - GPU tests, config 2 hold mode, 70B, transparent 70B.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_packing_gpu.py tests/test_managed_mode_gpu.py tests/test_model_gpu.py > gpurun_out/r5/p_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/r5/p_tests.log; exit 1; }
tail -2 gpurun_out/r5/p_tests.log
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('stream_stats_per_step'))"; }
run_b() {
  local tag=$1; shift
  timeout -k 10 500 python -u bench.py --no-aux "$@" > gpurun_out/r5/p_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/p_$tag.log; return 1; }
  summ gpurun_out/r5/p_$tag.log $tag
}
run_tm() {
  local tag=$1; shift
  env "$@" timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/p_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/p_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/p_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; p=a.get('pack',{}); print('$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'], {k: p.get(k) for k in ('packed_blocks','decodes_per_step','expansions')})"
}
run_b c2_off --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b c2_off_b --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b 70b --steps 6 --warmup 4 && \
run_tm tm_a OGKM_PACK=1 && run_tm tm_b OGKM_PACK=1 || exit 1
echo ALL_OK
