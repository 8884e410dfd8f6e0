#!/bin/bash
# Round 5 (k): transparent 70B with packed host copies - staging on 2 SDMA
# engines vs direct host decode, runtime spread on / off, raw baseline.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
run_tm() {  # $1 = tag, rest = env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 3 > gpurun_out/r5/k_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/k_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/k_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; p=a.get('pack',{}); print('$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'], {k: p.get(k) for k in ('packed_blocks','decodes_per_step','expansions')})"
}
run_tm stage2 OGKM_PACK=1 && \
run_tm direct OGKM_PACK=1 RT_ANS_STAGE_MB=0 && \
run_tm stage2_nospread OGKM_PACK=1 RT_PERF_SPREAD_ENABLE=0 && \
run_tm raw_nospread OGKM_PACK=0 RT_PERF_SPREAD_ENABLE=0 || exit 1
echo ALL_OK
