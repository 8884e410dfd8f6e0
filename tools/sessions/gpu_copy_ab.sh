#!/bin/bash
# Copy-kernel variants vs the hipMemcpyAsync default under the 70B bench: plain (not non-temporal)
# source loads at 16 and 32 workgroups. Each run time-limited; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
RT_COPY_ENGINE=0 RT_COPY_NT_LOADS=0 timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-aux > gpurun_out/ab_plain16.log 2>&1 || { echo P16_FAIL; tail -20 gpurun_out/ab_plain16.log; exit 1; }
grep '^{' gpurun_out/ab_plain16.log | cut -c1-170
RT_COPY_ENGINE=0 RT_COPY_NT_LOADS=0 RT_COPY_WORKGROUPS=32 timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-aux > gpurun_out/ab_plain32.log 2>&1 || { echo P32_FAIL; tail -20 gpurun_out/ab_plain32.log; exit 1; }
grep '^{' gpurun_out/ab_plain32.log | cut -c1-170
