#!/bin/bash
# One GPU session: streaming microbench, GPU tests, smoke, and the 70B bench
# (packed + raw host copies) with a rocprofv3 kernel trace of the packed run.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python tools/bench_stream.py > gpurun_out/stream.log 2>&1 || { echo STREAM_FAIL; tail -20 gpurun_out/stream.log; exit 1; }
grep '^{' gpurun_out/stream.log
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo GPU_TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 700 python bench.py --steps 5 --warmup 2 --verbose > gpurun_out/bench70b.log 2>&1 || { echo B70_FAIL; tail -30 gpurun_out/bench70b.log; exit 1; }
grep '^{' gpurun_out/bench70b.log
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof70b -o k -- python $R/bench.py --steps 3 --warmup 1 --no-aux > gpurun_out/bench70b_prof.log 2>&1 || { echo B70PROF_FAIL; tail -30 gpurun_out/bench70b_prof.log; exit 1; }
grep '^{' gpurun_out/bench70b_prof.log
timeout -k 10 600 python bench.py --steps 4 --warmup 2 --weights bf16 --no-aux > gpurun_out/bench70b_bf16.log 2>&1 || { echo B70BF16_FAIL; tail -30 gpurun_out/bench70b_bf16.log; exit 1; }
grep '^{' gpurun_out/bench70b_bf16.log
