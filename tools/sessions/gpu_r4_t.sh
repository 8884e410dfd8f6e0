#!/bin/bash
# Round 4: config-2 timed-step kernel trace + PMC (FETCH_SIZE, TA_BUSY), 70B headline kernel trace.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
rm -rf gpurun_out/r4/prof_c2b gpurun_out/r4/pmc_c2 gpurun_out/r4/prof_70b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_c2b -o run -- python bench.py --model llama3-8b --oversub 1 --steps 20 --warmup 3 --no-aux > gpurun_out/r4/t_c2.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r4/t_c2.log; exit 1; }
grep '^{' gpurun_out/r4/t_c2.log | cut -c1-200
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr -d gpurun_out/r4/pmc_c2 -o pmc -- python bench.py --model llama3-8b --oversub 1 --steps 5 --warmup 2 --no-aux > gpurun_out/r4/t_pmc.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/r4/t_pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4/pmc_c2 > gpurun_out/r4/t_pmc_summary.txt 2>&1; head -30 gpurun_out/r4/t_pmc_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_70b -o run -- python bench.py --steps 6 --warmup 3 --no-aux > gpurun_out/r4/t_70b.log 2>&1 || { echo PROF70_FAIL; tail -20 gpurun_out/r4/t_70b.log; exit 1; }
grep '^{' gpurun_out/r4/t_70b.log | cut -c1-200
echo ALL_OK
