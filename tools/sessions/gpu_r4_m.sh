#!/bin/bash
# Round 4: ranked victim cache + reuse cooldown (next-use eviction): stock-torch 70B / 8B, planner off.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 600 python -u bench.py --torch-managed --model $model --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/m_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/m_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/m_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], {k: a.get(k) for k in ('htd_gb_per_step','dth_gb_per_step','link_gbps','vmm_remaps','host_ms_per_step')})"
}
run_off() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --planner off --steps 6 --warmup 3 --no-aux > gpurun_out/r4/m_off_$tag.log 2>&1 || { echo OFF_FAIL $tag; tail -30 gpurun_out/r4/m_off_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/m_off_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('off_$tag', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['evictions'])"
}
run_tm 70b llama3-70b X=1 && run_tm 70b_cool8 llama3-70b RT_ARENA_REUSE_COOLDOWN=8 && run_tm 8b llama3-8b X=1 || exit 1
run_off cool0 X=1 && run_off cool8 RT_ARENA_REUSE_COOLDOWN=8 && run_off cool16 RT_ARENA_REUSE_COOLDOWN=16 || exit 1
echo ALL_OK
