#!/bin/bash
# Round 4: asynchronous prefetch worker for the transparent mode - GPU suite,
# stock-torch managed 8B (async on / off, lookahead sweep), host profile.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4/d_gpu.log 2>&1 || { echo GPU_FAIL; tail -60 gpurun_out/r4/d_gpu.log; exit 1; }
tail -2 gpurun_out/r4/d_gpu.log
for v in "OGKM_MANAGED_LOOKAHEAD_MB=-1" "OGKM_MANAGED_LOOKAHEAD_MB=256" "OGKM_MANAGED_LOOKAHEAD_MB=2048" "RT_TORCH_ASYNC_PREFETCH=0"; do
  env $v timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r4/d_tm.log 2>&1 || { echo TM_FAIL $v; tail -30 gpurun_out/r4/d_tm.log; exit 1; }
  grep '^{' gpurun_out/r4/d_tm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$v', d['value'], d['ms_per_step'], 'htd', a['htd_gb_per_step'], 'dth', a['dth_gb_per_step'], 'link', a['link_gbps'], 'remaps', a['vmm_remaps'], 'flushes', a['tlb_flushes'])"
  cp gpurun_out/r4/d_tm.log "gpurun_out/r4/d_tm_$(echo $v | tr '=' '_').log"
done
timeout -k 10 300 python -u tools/prof_torch_managed.py --steps 2 > gpurun_out/r4/d_prof_tm.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/r4/d_prof_tm.log; exit 1; }
head -25 gpurun_out/r4/d_prof_tm.log
echo ALL_OK
