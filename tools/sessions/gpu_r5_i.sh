#!/bin/bash
# Round 5 (i): VMM multi-chunk mapping probe; config 2 planner off vs static
# after the batched lease fast path / shared release event.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5 build
hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_offset.hip -lhsa-runtime64 -o build/probe_vmm_offset > /dev/null 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 60 ./build/probe_vmm_offset > gpurun_out/r5/i_probe.txt 2>&1 || { echo PROBE_FAIL; cat gpurun_out/r5/i_probe.txt; exit 1; }
cat gpurun_out/r5/i_probe.txt
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$2', d['value'], d['ms_per_step'], d['config']['planner'], a.get('stream_stats_per_step'))"; }
run_b() {
  local tag=$1; shift
  timeout -k 10 500 python -u bench.py --no-aux "$@" > gpurun_out/r5/i_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/i_$tag.log; return 1; }
  summ gpurun_out/r5/i_$tag.log $tag
}
run_b c2_off --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 && \
run_b c2_static --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --planner static && \
run_b c2_off_b --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 || exit 1
echo ALL_OK
