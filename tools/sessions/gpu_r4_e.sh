#!/bin/bash
# Round 4: host-time breakdown of the stock-torch managed 8B (inline prefetch),
# unmap / batch variants, then the stock-torch 70B under the transparent mode.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_tm() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r4/e_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/e_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/e_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], 'htd', a['htd_gb_per_step'], 'dth', a['dth_gb_per_step'], 'link', a['link_gbps'], 'remaps', a['vmm_remaps'], 'flushes', a['tlb_flushes'], 'host', a['host_ms_per_step'])"
}
run_tm default X=1 && run_tm lazy RT_STABLE_LAZY_UNMAP=1 && run_tm batch8 RT_STABLE_BATCH_BLOCKS=8 && run_tm batch128 RT_STABLE_BATCH_BLOCKS=128 || exit 1
timeout -k 10 900 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 2 > gpurun_out/r4/e_tm70.log 2>&1 || { echo TM70_FAIL; tail -30 gpurun_out/r4/e_tm70.log; exit 1; }
grep '^{' gpurun_out/r4/e_tm70.log
echo ALL_OK
