#!/bin/bash
# Round 4: direct-epilogue tests + config-2 A/B, then the planner-off window variants (gpu_r4_i.sh).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_dgemm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fixup or depths or numerics" > gpurun_out/r4/j_fix_tests.log 2>&1 || { echo FIXTEST_FAIL; tail -30 gpurun_out/r4/j_fix_tests.log; exit 1; }
tail -2 gpurun_out/r4/j_fix_tests.log
for f in 1 0 1 0; do
  OGKM_DGEMM_DIRECT=$f timeout -k 10 300 python bench.py --model llama3-8b --oversub 1 --steps 30 --warmup 5 --no-aux > gpurun_out/r4/j_c2_direct$f.log 2>&1 || { echo C2_FAIL; tail -20 gpurun_out/r4/j_c2_direct$f.log; exit 1; }
  echo "direct=$f $(grep '^{' gpurun_out/r4/j_c2_direct$f.log | cut -c1-160)"
done
timeout -k 10 120 ./tools/bin/probe_vmm_rocr_path > gpurun_out/r4/j_probe_rocr.txt 2>&1 && cat gpurun_out/r4/j_probe_rocr.txt && bash tools/gpu_r4_i.sh
