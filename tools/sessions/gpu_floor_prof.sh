set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
rm -rf gpurun_out/prof_floor
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_floor -o k -- python $R/bench.py --steps 3 --warmup 1 --no-aux --oversub 1.0 ${BENCH_ARGS} > gpurun_out/floor_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/floor_prof.log; exit 1; }
grep '^{' gpurun_out/floor_prof.log | cut -c1-200
python tools/trace_gaps.py gpurun_out/prof_floor --last-ms 1000 --copy NONE > gpurun_out/floor_kernels.txt 2>&1; tail -16 gpurun_out/floor_kernels.txt
