#!/bin/bash
# Round 5 (v): fused-combine latency-shaped attention (k_attn_decode_fl): numerics
# (auto / forced on / forced off), rates per shape, tp8 kernel trace; host-VMM probe.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
for fl in -1 1 0; do
  OGKM_ATTN_FL=$fl timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_fused.py -k "attention and not kv_rate" > gpurun_out/r5/v_attn_tests_$fl.log 2>&1 || { echo ATTN_TESTS_FAIL $fl; tail -30 gpurun_out/r5/v_attn_tests_$fl.log; exit 1; }
  echo "fl $fl tests: $(tail -1 gpurun_out/r5/v_attn_tests_$fl.log)"
  OGKM_ATTN_FL=$fl timeout -k 10 120 python -u -m pytest -q -s --timeout 100 --timeout-method thread tests/test_fused.py -k "kv_rate" > gpurun_out/r5/v_rate_$fl.log 2>&1; echo "fl $fl rate rc=$?"; grep "TB/s of KV" gpurun_out/r5/v_rate_$fl.log
  OGKM_ATTN_FL=$fl timeout -k 10 180 python -u tools/bench_attn.py > gpurun_out/r5/v_attn_$fl.txt 2>&1 || { echo ATTN_FAIL $fl; tail -20 gpurun_out/r5/v_attn_$fl.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r5/v_attn_$fl.txt | sed "s/^/fl $fl /"
done
cd /tmp && SHAPE=70b-tp8 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5/v_prof_tp8 -o attn -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py > $GRAFT_REPO_ROOT/gpurun_out/r5/v_prof_tp8.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r5/v_prof_tp8.log; exit 1; }
cd $GRAFT_REPO_ROOT
mkdir -p build
hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_host.hip -lhsa-runtime64 -o build/probe_vmm_host > gpurun_out/r5/v_probe_build.log 2>&1 || { echo PROBE_BUILD_FAIL; cat gpurun_out/r5/v_probe_build.log; exit 1; }
timeout -k 10 120 ./build/probe_vmm_host > gpurun_out/r5/v_probe_vmm_host.txt 2>&1; prc=$?; echo "probe rc=$prc"; cat gpurun_out/r5/v_probe_vmm_host.txt
echo ALL_OK
