#!/bin/bash
# 405B tp8-shard three-tier regression bisect: copy engine and weight/KV format; 8B resident raw formats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/bisect.log
run() {
  echo "== $*" >> gpurun_out/bisect.log
  timeout -k 10 300 "$@" >> gpurun_out/bisect.log 2>&1 || { echo "FAIL $*"; tail -8 gpurun_out/bisect.log; exit 1; }
  grep '^{' gpurun_out/bisect.log | tail -1 | cut -c1-130
  grep 'one step' gpurun_out/bisect.log | tail -1
}
B="python bench.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 2 --warmup 1 --no-aux --verbose"
run $B
run env RT_COPY_ENGINE=0 $B
run $B --weights bf11 --kv-format bf11
run python bench.py --model llama3-8b --oversub 1.0 --steps 5 --warmup 2 --no-aux --weights bf16 --kv-format bf16
