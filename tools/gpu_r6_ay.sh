#!/bin/bash
# round 6 (ay): final-build numbers for config 2 (8B HBM-resident, framework allocator) and the transparent 70B
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 500 python -u bench.py --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r6/ay_c2.log 2>&1 || { echo C2_FAIL; tail -5 gpurun_out/r6/ay_c2.log; exit 1; }
grep '"metric"' gpurun_out/r6/ay_c2.log | cut -c1-220
timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/ay_tm70b.log 2>&1 || { echo TM_FAIL; tail -5 gpurun_out/r6/ay_tm70b.log; exit 1; }
grep '"metric"' gpurun_out/r6/ay_tm70b.log | cut -c1-220
