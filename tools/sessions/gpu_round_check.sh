# Round check on one GPU: GPU tests, smoke, 70B headline; then rocprof of the
# page-list kernel (LDS) and a marker (roctx) trace of a short 8B oversubscribed run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_verify.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pagelist -o run -- python -m pytest tests/test_gpu_runtime.py -q -k fragmented > gpurun_out/prof_pagelist.log 2>&1 || { echo PROF_PL_FAIL; tail -20 gpurun_out/prof_pagelist.log; exit 1; }
timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace -d gpurun_out/prof_markers -o run -- python bench.py --model llama3-8b --oversub 1.5 --steps 2 --warmup 1 --no-aux > gpurun_out/prof_markers.log 2>&1 || { echo PROF_MK_FAIL; tail -20 gpurun_out/prof_markers.log; exit 1; }
grep '^{' gpurun_out/prof_markers.log | cut -c1-200
