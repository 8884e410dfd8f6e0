#!/bin/bash
# Round 4: transparent mode - managed-range size threshold (activations below it stay plain HBM allocations).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 500 python -u bench.py --torch-managed --model $model --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/mm_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/mm_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/mm_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['faulted_ops'], a['ring_per_step'], a['host_ms_per_step'])"
}
run_tm 70b_min4 llama3-70b OGKM_MANAGED_MIN_MB=4 && run_tm 70b_min16 llama3-70b OGKM_MANAGED_MIN_MB=16 && run_tm 8b_min4 llama3-8b OGKM_MANAGED_MIN_MB=4 || exit 1
echo ALL_OK
