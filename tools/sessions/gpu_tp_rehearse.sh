#!/bin/bash
# GPU tests + smoke, then per-rank rehearsal of the multi-GPU bench on one GPU (--simulate-tp: the
# TP rank-0 shard of an N-GPU job) with the default formats/engine, and a longer 405B shard run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
: > gpurun_out/rehearse.log
run() {
  echo "== $*" >> gpurun_out/rehearse.log
  timeout -k 10 300 "$@" >> gpurun_out/rehearse.log 2>&1 || { echo "FAIL $*"; tail -8 gpurun_out/rehearse.log; exit 1; }
  grep '^{' gpurun_out/rehearse.log | tail -1 | cut -c1-130
  grep 'one step' gpurun_out/rehearse.log | tail -1
}
run python bench.py --simulate-tp 8 --steps 5 --warmup 2 --no-aux --verbose
run python bench.py --simulate-tp 4 --steps 5 --warmup 2 --no-aux --verbose
run python bench.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 5 --warmup 3 --no-aux --verbose
