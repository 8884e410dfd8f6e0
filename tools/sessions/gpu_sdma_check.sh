# SDMA ring engine on the GPU: tests, smoke, 70B headline, kernel trace of a short run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_verify.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sdma -o run -- python bench.py --steps 3 --warmup 1 --no-aux > gpurun_out/prof_sdma.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_sdma.log; exit 1; }
grep '^{' gpurun_out/prof_sdma.log | cut -c1-160
find gpurun_out/prof_sdma -name "*kernel_stats*" | head -3
