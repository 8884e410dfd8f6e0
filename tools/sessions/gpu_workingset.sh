#!/bin/bash
# planner-off 70B 2x: refault-protected workingset with spread admission (+ a larger prefetch window).
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --planner off --steps 4 --warmup 3 --no-aux > gpurun_out/ws_$tag.log 2>&1 || { echo WS_FAIL $tag; tail -5 gpurun_out/ws_$tag.log; exit 1; }
  grep '^{' gpurun_out/ws_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], 'tok/s', d['ms_per_step'], 'ms', 'link', d['aux']['link_gbps_per_gpu'], 'GB/step', round(d['aux']['link_gbps_per_gpu'] * d['ms_per_step'] / 1000, 2), 'evictions', d['aux']['evictions'])"
}
run spread95 RT_PERF_WORKINGSET_ACTIVE_PCT=95
run spread95_w2g RT_PERF_WORKINGSET_ACTIVE_PCT=95 OGKM_WINDOW_MB=2048
run spread97 RT_PERF_WORKINGSET_ACTIVE_PCT=97
