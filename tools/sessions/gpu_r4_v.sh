#!/bin/bash
# Round 4: stock-torch 70B under ogkm.managed() - async prefetch worker and lookahead variants.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_tm() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/v_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/v_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/v_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
}
run_tm async RT_TORCH_ASYNC_PREFETCH=1 && run_tm la4g OGKM_MANAGED_LOOKAHEAD_MB=4096 && run_tm la20g OGKM_MANAGED_LOOKAHEAD_MB=20480 || exit 1
echo ALL_OK
