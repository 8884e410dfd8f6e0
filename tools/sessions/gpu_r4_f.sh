#!/bin/bash
# Round 4: home-chunk placement (eager / lazy unmap) for the stock-torch managed
# decode, the 70B under the transparent mode, planner off and the headline.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 900 python -u bench.py --torch-managed --model $model --oversub 2 --steps 4 --warmup 3 > gpurun_out/r4/f_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/f_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/f_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], 'htd', a['htd_gb_per_step'], 'dth', a['dth_gb_per_step'], 'link', a['link_gbps'], 'remaps', a['vmm_remaps'], 'flushes', a['tlb_flushes'], 'host', a['host_ms_per_step'])"
}
run_tm 8b_eager llama3-8b X=1 && run_tm 8b_lazy llama3-8b RT_STABLE_LAZY_UNMAP=1 || exit 1
timeout -k 10 600 python -u bench.py --planner off --steps 8 --warmup 3 --no-aux --verbose > gpurun_out/r4/f_off.log 2>&1 || { echo OFF_FAIL; tail -30 gpurun_out/r4/f_off.log; exit 1; }
grep "one step" gpurun_out/r4/f_off.log
grep '^{' gpurun_out/r4/f_off.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('planner_off', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['evictions'])"
run_tm 70b_lazy llama3-70b RT_STABLE_LAZY_UNMAP=1 || exit 1
echo ALL_OK
