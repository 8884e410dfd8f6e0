#!/bin/bash
# k_dgemm_pipe unit sweep vs k_dgemm<RAW,2>; managed-mode prefetch lookahead sweep.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
S8="6144x4096,4096x4096,28672x4096,4096x14336"
run() {  # tag variants env...
  local tag=$1 v=$2; shift 2
  env "$@" SHAPES=$S8 VARIANTS="$v" timeout -k 10 120 python -u tools/bench_dgemm.py > gpurun_out/r3/sw2_8b_$tag.jsonl 2>&1 || return 1
  env "$@" VARIANTS="$v" timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/sw2_70b_$tag.jsonl 2>&1 || return 1
  echo "$tag 8b $(grep '^{' gpurun_out/r3/sw2_8b_$tag.jsonl | cut -c1-250)"
  echo "$tag 70b $(grep '^{' gpurun_out/r3/sw2_70b_$tag.jsonl | cut -c1-250)"
}
run split768 "raw:2" OGKM_DGEMM_UNITS=768 || exit 1
for u in 512 768 1024 1536 2048; do run pipe$u "pipe:2" OGKM_DGEMM_UNITS_PIPE=$u || exit 1; done
for la in 256 512 1024 2048; do
  OGKM_MANAGED_LOOKAHEAD_MB=$la timeout -k 10 300 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 2 --warmup 1 > gpurun_out/r3/tm_la$la.log 2>&1 || { echo TM_FAIL $la; tail -5 gpurun_out/r3/tm_la$la.log; exit 1; }
  echo "la $la $(grep '^{' gpurun_out/r3/tm_la$la.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); a=d["aux"]; print(d["value"], d["ms_per_step"], a["htd_gb_per_step"], a["dth_gb_per_step"], a["link_gbps"])')"
done
echo ALL_OK
