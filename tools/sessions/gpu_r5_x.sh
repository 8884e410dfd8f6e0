#!/bin/bash
# Round 5 (x): transparent 70B - staging engines / staging size sweep on the
# merged + overlapped H2D ring.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
tm() {
  local tag=$1; shift
  env "$@" OGKM_PACK=1 timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r5/x_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r5/x_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r5/x_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm $tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
}
tm eng_f RT_ANS_STAGE_ENGINES=0xF && tm stage128 RT_ANS_STAGE_MB=128 RT_RING_MERGE_PACKED_MB=64 && tm eng_1 RT_ANS_STAGE_ENGINES=0x1 && tm default || exit 1
echo ALL_OK
