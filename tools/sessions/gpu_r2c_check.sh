#!/bin/bash
# Full GPU suite + smoke + headline, then the tp8-shard step-0 transient check.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_verify.sh || exit 1
timeout -k 10 400 python -u tools/diag_transient.py --model llama3-70b --simulate-tp 8 --steps 4 > gpurun_out/r2c_diag_tp8.log 2>&1; rc=$?
grep -E "^step [0-9]+: host|^step [0-9]+: [0-9.]+ ms|transient" gpurun_out/r2c_diag_tp8.log | cut -c1-160
exit $rc
