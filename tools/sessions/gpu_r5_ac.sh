#!/bin/bash
# Round 5 (ac): packing while GPU copies are leased - GPU numerics, transparent 70B
# census; long context under planner off with a wider window / more run-ahead.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_packing_gpu.py tests/test_managed_mode_gpu.py > gpurun_out/r5/ac_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r5/ac_tests.log; exit 1; }
tail -1 gpurun_out/r5/ac_tests.log
OGKM_TM_CENSUS=1 OGKM_PACK=1 timeout -k 10 700 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/ac_tm_census.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r5/ac_tm_census.log; exit 1; }
grep '^{' gpurun_out/r5/ac_tm_census.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step']); print(a['block_census']['blocks']); print(a['pack'])"
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('link_gbps_per_gpu'), a.get('ring_per_step'), {k: (a.get('stream_stats_per_step') or {}).get(k) for k in ('prefetch_ms','ahead_wait_ms','wait_ms','use_ms')})"; }
lc() {
  local tag=$1; shift
  env "$@" timeout -k 10 700 python -u bench.py --no-aux --context 32768 --batch 8 --kv-tiering --steps 3 --warmup 2 > gpurun_out/r5/ac_$tag.log 2>&1 || { echo LC_FAIL $tag; tail -30 gpurun_out/r5/ac_$tag.log; return 1; }
  summ gpurun_out/r5/ac_$tag.log $tag
}
lc win4g OGKM_WINDOW_MB=4096 && lc runahead3 OGKM_RUNAHEAD=3 OGKM_MAX_AHEAD=64 && lc nowaitissued RT_RING_WAIT_ISSUED=0 OGKM_MAX_AHEAD=64 || exit 1
echo ALL_OK
