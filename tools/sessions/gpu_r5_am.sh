#!/bin/bash
# Round 5 (am): refill-cost-aware next-use victims on the transparent 70B
# (arena_cheap_refill_bias_pct 0 / 50 / 100).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tm() {
  local tag=$1; shift
  env "$@" OGKM_PACK=1 timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/am_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/am_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/am_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm $tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['ring_per_step'])"
}
tm bias100 RT_ARENA_CHEAP_REFILL_BIAS_PCT=100 && tm bias0 RT_ARENA_CHEAP_REFILL_BIAS_PCT=0 && tm bias50 RT_ARENA_CHEAP_REFILL_BIAS_PCT=50 || exit 1
echo ALL_OK
