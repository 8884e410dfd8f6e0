#!/bin/bash
# Round 4: planner-off variants (gpu_r4_i.sh), then the ROCr remap probe (timing, then HIP copies on ROCr-only VAs).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
bash tools/gpu_r4_i.sh || exit 1
timeout -k 10 120 ./tools/bin/probe_vmm_rocr_path 0 > gpurun_out/r4/k_probe_rocr0.txt 2>&1 || { echo PROBE0_FAIL; tail -5 gpurun_out/r4/k_probe_rocr0.txt; exit 1; }
grep -v "^step" gpurun_out/r4/k_probe_rocr0.txt
timeout -k 10 120 ./tools/bin/probe_vmm_rocr_path 1 > gpurun_out/r4/k_probe_rocr1.txt 2>&1 || { echo PROBE1_FAIL; tail -5 gpurun_out/r4/k_probe_rocr1.txt; exit 1; }
grep -v "^step" gpurun_out/r4/k_probe_rocr1.txt
