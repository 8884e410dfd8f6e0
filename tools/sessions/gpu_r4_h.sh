#!/bin/bash
# Round 4: split-K fixup tests + config-2 profile / A-B, 70B stock-torch managed with the age-based persistence rule, 8B check.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_dgemm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fixup or depths" > gpurun_out/r4/h_fix_tests.log 2>&1 || { echo FIXTEST_FAIL; tail -30 gpurun_out/r4/h_fix_tests.log; exit 1; }
tail -2 gpurun_out/r4/h_fix_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_c2 -o run -- python bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r4/h_c2.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r4/h_c2.log; exit 1; }
grep '^{' gpurun_out/r4/h_c2.log | cut -c1-200
for f in 1 0 1 0; do
  OGKM_DGEMM_FIXUP=$f timeout -k 10 300 python bench.py --model llama3-8b --oversub 1 --steps 30 --warmup 5 --no-aux > gpurun_out/r4/h_c2_fix$f.log 2>&1 || { echo C2_FAIL; tail -20 gpurun_out/r4/h_c2_fix$f.log; exit 1; }
  echo "fixup=$f $(grep '^{' gpurun_out/r4/h_c2_fix$f.log | cut -c1-160)"
done
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 900 python -u bench.py --torch-managed --model $model --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/h_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/h_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/h_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('$tag', d['value'], d['ms_per_step'], {k: a.get(k) for k in ('htd_gb_per_step','dth_gb_per_step','link_gbps','evictions','vmm_remaps','faulted_ops','prefetches','trace_len','hinted_ops','trace_misses','ops','host_ms_per_step')})"
}
run_tm 70b llama3-70b X=1 && run_tm 8b llama3-8b X=1 || exit 1
echo ALL_OK
