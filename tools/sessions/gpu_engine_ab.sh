#!/bin/bash
# A/B of the H2D engine under the 70B ans bench: SDMA (RT_COPY_ENGINE=1) vs copy kernels at fewer workgroups.
# Each run time-limited; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
RT_COPY_ENGINE=1 timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-aux --weights ans > gpurun_out/ab_sdma.log 2>&1 || { echo SDMA_FAIL; tail -20 gpurun_out/ab_sdma.log; exit 1; }
grep '^{' gpurun_out/ab_sdma.log | cut -c1-200
export RT_COPY_ENGINE=1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sdma -o k -- python $R/bench.py --steps 3 --warmup 1 --no-aux --weights ans > gpurun_out/prof_sdma.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_sdma.log; exit 1; }
unset RT_COPY_ENGINE
RT_COPY_WORKGROUPS=8 timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-aux --weights ans > gpurun_out/ab_wg8.log 2>&1 || { echo WG8_FAIL; tail -20 gpurun_out/ab_wg8.log; exit 1; }
grep '^{' gpurun_out/ab_wg8.log | cut -c1-200
