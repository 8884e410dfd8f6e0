#!/bin/bash
# Round 4: pipelined DMA ring worker - GPU tests, then static / planner off (+ deeper window) / stock-torch 70B and 8B.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_managed_mode_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/o_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error" gpurun_out/r4/o_tests.log | head; tail -15 gpurun_out/r4/o_tests.log; exit 1; }
tail -1 gpurun_out/r4/o_tests.log
run_b() {  # $1 = tag, $2 = planner, rest = env
  local tag=$1 pl=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --planner $pl --steps 4 --warmup 3 --no-aux > gpurun_out/r4/o_$tag.log 2>&1 || { echo RUN_FAIL $tag; tail -30 gpurun_out/r4/o_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/o_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['aux']['traffic_per_step_gb']['pcie_measured'], d['aux']['ring_per_step'])"
}
run_b static static X=1 && run_b off off X=1 && run_b off_deep off OGKM_WINDOW_MISSING=1 OGKM_MAX_AHEAD=12 OGKM_WINDOW_MB=1024 || exit 1
run_tm() {  # $1 = tag, $2 = model, rest = env
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 600 python -u bench.py --torch-managed --model $model --oversub 2 --steps 3 --warmup 3 > gpurun_out/r4/o_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 gpurun_out/r4/o_tm_$tag.log; return 1; }
  grep '^{' gpurun_out/r4/o_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm_$tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['dth_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
}
run_tm 70b llama3-70b X=1 && run_tm 8b llama3-8b X=1 || exit 1
echo ALL_OK
