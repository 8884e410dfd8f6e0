set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dgemm.py tests/test_gpu_runtime.py -m gpu -q -rA -s --timeout 120 --timeout-method thread > gpurun_out/dgemm_tests.log 2>&1; rc=$?
grep -E "passed|failed|Error" gpurun_out/dgemm_tests.log | tail -5
true
timeout -k 10 300 python tools/bench_dgemm.py > gpurun_out/bench_dgemm.log 2>&1; rc=$?
cat gpurun_out/bench_dgemm.log | tail -12

export TMPDIR=/tmp
VARIANTS=bf11:2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d $PWD/gpurun_out/pmc_dgemm -o pmc -- python tools/bench_dgemm.py > gpurun_out/pmc_dgemm.log 2>&1
echo pmc rc=$?
exit 0
