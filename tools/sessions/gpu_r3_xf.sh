#!/bin/bash
# GEMM access-pattern probe (fragment-ordered activations) + config 2 deferred
# epilogue A/B, alternating runs on one box.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3 /tmp/pb
hipcc --offload-arch=gfx950 -O3 tools/probe_gemm_pattern.hip -o /tmp/pb/pgp && timeout -k 10 200 /tmp/pb/pgp > gpurun_out/r3/gemm_pattern2.jsonl 2>&1 || { echo PGP_FAIL; exit 1; }
for F in 1 0 1 0; do
  OGKM_FUSE_EPI=$F timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/c2ab_$F.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/c2ab_$F.log; exit 1; }
  echo "fuse $F $(grep '^{' gpurun_out/r3/c2ab_$F.log | cut -c1-160)"
done
echo ALL_OK
