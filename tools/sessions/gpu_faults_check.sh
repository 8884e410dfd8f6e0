# Device fault path on the GPU: GET/PUT ring stress, fault gate + replay, table shootdown.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_faults.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_faults.log 2>&1; rc=$?
tail -8 gpurun_out/gpu_faults.log
exit $rc
