# Compute floor of the decode step: everything HBM-resident (oversub 1.0), with a kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-aux --oversub 1.0 > gpurun_out/floor.log 2>&1 || { echo FLOOR_FAIL; tail -20 gpurun_out/floor.log; exit 1; }
grep '^{' gpurun_out/floor.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_floor -o k -- python $R/bench.py --steps 3 --warmup 1 --no-aux --oversub 1.0 > gpurun_out/floor_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/floor_prof.log; exit 1; }
python tools/trace_gaps.py gpurun_out/prof_floor --last-ms 1500 --copy NONE > gpurun_out/floor_kernels.txt 2>&1; tail -18 gpurun_out/floor_kernels.txt
