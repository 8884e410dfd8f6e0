#!/bin/bash
# Per-rank rehearsal of the N-GPU bench on one GPU (--simulate-tp N = TP rank-0 shard) after the
# unit-size floor; GPU tests first. Each step time-limited; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head; exit 1; }
tail -1 gpurun_out/gpu_tests.log
: > gpurun_out/rehearse2.log
run() {
  echo "== $*" >> gpurun_out/rehearse2.log
  timeout -k 10 300 "$@" >> gpurun_out/rehearse2.log 2>&1 || { echo "FAIL $*"; tail -8 gpurun_out/rehearse2.log; exit 1; }
  grep '^{' gpurun_out/rehearse2.log | tail -1 | cut -c1-130
  grep 'one step' gpurun_out/rehearse2.log | tail -1
}
for n in 8 4 2; do run python bench.py --simulate-tp $n --steps 5 --warmup 3 --no-aux --verbose; done
