#!/bin/bash
# Round 4: stable-VA remaps through ROCr (placeholder HIP view): managed GPU tests, stock-torch 8B / 70B,
# then a planner-off copy trace (SDMA copy sizes / gaps).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_managed_mode_gpu.py tests/test_allocator.py tests/test_gpu_runtime.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/l_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|error" gpurun_out/r4/l_tests.log | head -20; tail -20 gpurun_out/r4/l_tests.log; exit 1; }
tail -2 gpurun_out/r4/l_tests.log
grep -i "selftest\|self-test" gpurun_out/r4/l_tests.log | head -3
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 900 python -u bench.py --torch-managed --model $model --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/l_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/l_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/l_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], {k: a.get(k) for k in ('htd_gb_per_step','dth_gb_per_step','link_gbps','evictions','vmm_remaps','trace_misses','host_ms_per_step')})"
}
run_tm 8b llama3-8b X=1 && run_tm 8b_hip llama3-8b RT_VMM_ROCR_REMAP=0 && run_tm 70b llama3-70b X=1 || exit 1
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace -d gpurun_out/r4/prof_off -o run -- python bench.py --planner off --steps 3 --warmup 2 --no-aux > gpurun_out/r4/l_off_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r4/l_off_prof.log; exit 1; }
grep '^{' gpurun_out/r4/l_off_prof.log | cut -c1-200
echo ALL_OK
