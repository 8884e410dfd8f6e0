#!/bin/bash
# Round 5 (w): latency-shaped attention without the fused combine (A/B), the H2D
# ring's merged packed batches + overlapped staging halves (GPU numerics, then the
# transparent 70B step with and without them).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
for v in "1 0" "1 1" "0 1"; do
  set -- $v
  OGKM_ATTN_FL=$1 OGKM_ATTN_FL_FUSE=$2 timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/w_attn_$1$2.txt 2>&1 || { echo ATTN_FAIL $v; tail -20 gpurun_out/r5/w_attn_$1$2.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r5/w_attn_$1$2.txt | sed "s/^/fl $1 fuse $2 /"
done
OGKM_ATTN_FL=1 OGKM_ATTN_FL_FUSE=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused.py -k "attention and not kv_rate" > gpurun_out/r5/w_attn_tests.log 2>&1 || { echo ATTN_TESTS_FAIL; tail -30 gpurun_out/r5/w_attn_tests.log; exit 1; }
echo "fl nofuse tests: $(tail -1 gpurun_out/r5/w_attn_tests.log)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_packing_gpu.py tests/test_managed_mode_gpu.py > gpurun_out/r5/w_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r5/w_tests.log; exit 1; }
tail -1 gpurun_out/r5/w_tests.log
tm() {
  local tag=$1; shift
  env "$@" OGKM_PACK=1 timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/w_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/w_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/w_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm $tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'], a.get('pack'))"
}
tm new RT_RING_MERGE_PACKED_MB=24 && tm old RT_RING_MERGE_PACKED_MB=0 RT_RING_STAGE_OVERLAP=0 || exit 1
echo ALL_OK
