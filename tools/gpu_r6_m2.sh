#!/bin/bash
# round 6 (m2): headline bench, attention split A/B, config 2 (arena allocator
# default) + its kernel profile (kernel trace only).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/m_headline.log 2>&1 || { echo HEADLINE_FAIL; tail -30 gpurun_out/r6/m_headline.log; exit 1; }
grep '^{' gpurun_out/r6/m_headline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('headline', d['value'], d['ms_per_step'], a.get('link_gbps_per_gpu'), a.get('traffic_per_step_gb'))"
for sp in 0 64; do SPLIT=$sp timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/r6/m_attn_split$sp.log 2>&1 || exit 1; grep -v amdgpu.ids gpurun_out/r6/m_attn_split$sp.log | sed "s/^/split$sp /"; done
timeout -k 10 400 python -u bench.py --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r6/m_c2.log 2>&1 || { tail -10 gpurun_out/r6/m_c2.log; exit 1; }
grep '^{' gpurun_out/r6/m_c2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 default', d['value'], d['ms_per_step'], d['config'].get('torch_allocator'))"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/m_prof_c2 -o c2 -- python3 $R/bench.py --model llama3-8b --oversub 1.0 --steps 20 --warmup 5 --no-aux > $R/gpurun_out/r6/m_prof_c2.log 2>&1 || { echo PROF_FAIL; tail -5 $R/gpurun_out/r6/m_prof_c2.log; exit 1; }
echo ALL_OK
