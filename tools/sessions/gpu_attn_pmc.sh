#!/bin/bash
# Attention microbench + PMC passes (SQ, then TCC fetch) on the wave-split kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1; rc=$?
tail -2 gpurun_out/attn_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E )" gpurun_out/attn_tests.log | head -20; exit 1; }
timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_attn.txt
rm -rf gpurun_out/pmc_attn gpurun_out/pmc_attn2
ITERS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d $PWD/gpurun_out/pmc_attn -o pmc -- python tools/bench_attn.py > gpurun_out/pmc_attn.log 2>&1; echo pmc1 rc=$?
python tools/pmc_summary.py gpurun_out/pmc_attn --filter attn_decode_ws 2>&1 | head -40
ITERS=3 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VMEM_RD -d $PWD/gpurun_out/pmc_attn2 -o pmc -- python tools/bench_attn.py > gpurun_out/pmc_attn2.log 2>&1; echo pmc2 rc=$?
python tools/pmc_summary.py gpurun_out/pmc_attn2 --filter attn_decode_ws 2>&1 | head -30
