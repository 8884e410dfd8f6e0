#!/bin/bash
# Round 5 (l): transparent 70B with packing after the write-back fix (x2, spread
# on / off) + a kernel-trace profile of the packed transparent step.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/l_attn.txt 2>&1 && GRAPH=0 timeout -k 10 180 python -u tools/bench_attn.py >> gpurun_out/r5/l_attn.txt 2>&1 || { echo ATTN_FAIL; tail -20 gpurun_out/r5/l_attn.txt; exit 1; }
cat gpurun_out/r5/l_attn.txt | grep -v amdgpu.ids
run_tm() {  # $1 = tag, rest = env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/l_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/l_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/l_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; p=a.get('pack',{}); print('$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'], {k: p.get(k) for k in ('packed_blocks','decodes_per_step','expansions')})"
}
run_tm pack_a OGKM_PACK=1 && \
run_tm pack_nospread OGKM_PACK=1 RT_PERF_SPREAD_ENABLE=0 && \
run_tm pack_b OGKM_PACK=1 || exit 1
cd /tmp && timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5/prof_tm -o tm -- python3 $GRAFT_REPO_ROOT/bench.py --torch-managed --model llama3-70b --oversub 2 --steps 2 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r5/l_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r5/l_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/r5/prof_tm -name "*stats*" | head
echo ALL_OK
