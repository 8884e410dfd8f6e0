#!/bin/bash
# TLB-flush elision for stable-VA remaps: managed / stable-VA GPU tests, the
# managed round-trip bench and the stock-torch 8B managed-mode bench.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_runtime.py tests/test_managed_mode.py tests/test_allocator.py > gpurun_out/r3/tlb_tests.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r3/tlb_tests.log; exit 1; }
tail -2 gpurun_out/r3/tlb_tests.log
timeout -k 10 200 python -u tools/bench_managed.py --tensors 8 --mb 256 --arena-mb 1024 --iters 3 > gpurun_out/r3/tlb_bm.log 2>&1 || { echo BM_FAIL; tail -20 gpurun_out/r3/tlb_bm.log; exit 1; }
tail -1 gpurun_out/r3/tlb_bm.log | cut -c1-600
timeout -k 10 500 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 2 > gpurun_out/r3/tlb_tm8b.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r3/tlb_tm8b.log; exit 1; }
grep '^{' gpurun_out/r3/tlb_tm8b.log | cut -c1-1200
echo ALL_OK
