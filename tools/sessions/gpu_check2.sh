# GPU tests (incl. the dma-buf importer), then the transient-stall guard on the
# one-KV-head 70B tp8 shard (round-1 ADVICE: step 1 must not stall).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo GPU_TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 500 python -u tools/diag_transient.py --model llama3-70b --simulate-tp 8 --steps 4 > gpurun_out/diag_tp8.log 2>&1; rc=$?
grep -E "^step [0-9]+: [0-9.]+ ms|transient" gpurun_out/diag_tp8.log | cut -c1-120
exit $rc
