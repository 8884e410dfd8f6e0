#!/bin/bash
# Round 5 (e): 70B headline - runtime spread classes: online adaptation off/on,
# victim-cache rerank off/on, keep share (aux.spread has keep-class evictions per pass).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
summ() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux'].get('ring_per_step'), d['aux'].get('spread'))"; }
run_b() {  # $1 = tag, rest = env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 6 --warmup 4 --no-aux > gpurun_out/r5/e_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r5/e_$tag.log; return 1; }
  summ gpurun_out/r5/e_$tag.log $tag
}
mkdir -p build
hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_host.hip -lhsa-runtime64 -o build/probe_vmm_host > gpurun_out/r5/e_probe_build.log 2>&1 || { echo PROBE_BUILD_FAIL; cat gpurun_out/r5/e_probe_build.log; exit 1; }
timeout -k 10 120 ./build/probe_vmm_host > gpurun_out/r5/e_probe_vmm_host.txt 2>&1; prc=$?; echo "probe rc=$prc"; cat gpurun_out/r5/e_probe_vmm_host.txt
[ $prc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_tp2.py > gpurun_out/r5/e_tp2.log 2>&1; echo "tp2 rc=$?"; grep "max |diff|\|passed\|failed" gpurun_out/r5/e_tp2.log
run_b noadapt RT_PERF_SPREAD_ADAPT=0 && run_b noadapt_norerank RT_PERF_SPREAD_ADAPT=0 RT_ARENA_VICTIM_RERANK=0 && run_b noadapt_k94 RT_PERF_SPREAD_ADAPT=0 RT_PERF_SPREAD_KEEP_PCT=94 && run_b default X=1 || exit 1
echo ALL_OK
