#!/bin/bash
# Round-2b checks: new GPU tests (managed allocator, one-rank RCCL), step-0
# transient of the 70B tp8 shard and the 70B headline with --warmup 0 semantics
# (diag_transient), then the headline bench. Each step time-limited.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_runtime.py -k "rccl or managed or allocator" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r2b_tests.log 2>&1; rc=$?
tail -8 gpurun_out/r2b_tests.log
grep MANAGED_OK gpurun_out/r2b_tests.log | cut -c1-300
[ $rc -eq 0 ] || { echo TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/r2b_tests.log | head -30; exit 1; }
timeout -k 10 400 python -u tools/diag_transient.py --model llama3-70b --simulate-tp 8 --steps 4 > gpurun_out/r2b_diag_tp8.log 2>&1; rc=$?
grep -E "^step [0-9]+: [0-9.]+ ms|transient" gpurun_out/r2b_diag_tp8.log
[ $rc -eq 0 ] || { echo DIAG_TP8_FAIL; tail -5 gpurun_out/r2b_diag_tp8.log; }
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
timeout -k 10 500 python -u tools/diag_transient.py --model llama3-70b --steps 4 > gpurun_out/r2b_diag_70b.log 2>&1; rc=$?
grep -E "^step [0-9]+: [0-9.]+ ms|transient" gpurun_out/r2b_diag_70b.log
[ $rc -eq 0 ] || { echo DIAG_70B_FAIL; tail -5 gpurun_out/r2b_diag_70b.log; }
