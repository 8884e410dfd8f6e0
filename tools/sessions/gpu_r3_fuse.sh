#!/bin/bash
# Deferred GEMM epilogues: GPU tests, config 2 with and without, and the GEMM
# access-pattern probe.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3 /tmp/pb
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fused.py tests/test_model_gpu.py tests/test_dgemm.py > gpurun_out/r3/fuse_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r3/fuse_tests.log; exit 1; }
tail -2 gpurun_out/r3/fuse_tests.log
for F in 1 0; do
  OGKM_FUSE_EPI=$F timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 10 --warmup 3 --no-aux > gpurun_out/r3/c2_fuse$F.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/c2_fuse$F.log; exit 1; }
  echo "fuse $F"; grep '^{' gpurun_out/r3/c2_fuse$F.log | cut -c1-200
done
hipcc --offload-arch=gfx950 -O3 tools/probe_gemm_pattern.hip -o /tmp/pb/pgp && timeout -k 10 200 /tmp/pb/pgp > gpurun_out/r3/gemm_pattern.jsonl 2>&1 || { echo PGP_FAIL; exit 1; }
echo ALL_OK
