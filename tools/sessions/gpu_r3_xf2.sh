#!/bin/bash
# Fragment-ordered GEMM activations: GPU tests, cold GEMM sweep (row-major vs
# fragment x), config 2 A/B (alternating), 70B tp8-shard host step.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fused.py tests/test_model_gpu.py tests/test_dgemm.py > gpurun_out/r3/xf_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r3/xf_tests.log; exit 1; }
tail -2 gpurun_out/r3/xf_tests.log
S8="6144x4096,4096x4096,14336x4096,4096x14336,128256x4096"
for XF in 1 0; do
  XFRAG=$XF SHAPES=$S8 VARIANTS="pipe:0,pipe:4,pipe:50" timeout -k 10 200 python -u tools/bench_dgemm.py > gpurun_out/r3/xf8b_$XF.jsonl 2>&1 || { echo B8_FAIL; tail -20 gpurun_out/r3/xf8b_$XF.jsonl; exit 1; }
  XFRAG=$XF VARIANTS="pipe:0,pipe:4,pipe:50" timeout -k 10 300 python -u tools/bench_dgemm.py > gpurun_out/r3/xf70b_$XF.jsonl 2>&1 || { echo B70_FAIL; tail -20 gpurun_out/r3/xf70b_$XF.jsonl; exit 1; }
  echo "xfrag $XF"; grep '^{' gpurun_out/r3/xf8b_$XF.jsonl | cut -c1-330; grep '^{' gpurun_out/r3/xf70b_$XF.jsonl | cut -c1-300
done
for XF in 1 0 1 0; do
  OGKM_XFRAG=$XF timeout -k 10 300 python -u bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r3/c2xf_$XF.log 2>&1 || { echo C2_FAIL; tail -30 gpurun_out/r3/c2xf_$XF.log; exit 1; }
  echo "xfrag $XF $(grep '^{' gpurun_out/r3/c2xf_$XF.log | cut -c1-150)"
done
echo ALL_OK
