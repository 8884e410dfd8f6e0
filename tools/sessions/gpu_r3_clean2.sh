#!/bin/bash
# Managed-mode eviction experiments: clean-first eviction with / without the
# managed range cache, and the cache alone.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
run() {
  env "$@" timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r3/cl2.log 2>&1 || { echo TM_FAIL "$@"; tail -30 gpurun_out/r3/cl2.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/r3/cl2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); a=d["aux"]; print(d["value"], d["ms_per_step"], a["htd_gb_per_step"], a["dth_gb_per_step"], a["link_gbps"], a["tlb_flushes"])')"
}
run RT_TORCH_ALLOC_CACHE_MB=64
run RT_TORCH_ALLOC_CACHE_MB=128
run RT_TORCH_ALLOC_CACHE_MB=256
echo ALL_OK
