#!/bin/bash
# Load-time warm streaming pass: 70B default and 405B tp8-shard three-tier with a single warmup step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/warm.log
run() {
  echo "== $*" >> gpurun_out/warm.log
  timeout -k 10 300 "$@" >> gpurun_out/warm.log 2>&1 || { echo "FAIL $*"; tail -8 gpurun_out/warm.log; exit 1; }
  grep '^{' gpurun_out/warm.log | tail -1 | cut -c1-130
}
run python bench.py --steps 3 --warmup 1 --no-aux
run python bench.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 3 --warmup 1 --no-aux
