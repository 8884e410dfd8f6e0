set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof70b -o k -- python $R/bench.py --steps 3 --warmup 1 --no-aux ${BENCH_ARGS} > gpurun_out/bench70b_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/bench70b_prof.log; exit 1; }
grep '^{' gpurun_out/bench70b_prof.log
python tools/trace_gaps.py gpurun_out/prof70b --last-ms 2500 > gpurun_out/trace_gaps.txt 2>&1; cat gpurun_out/trace_gaps.txt
