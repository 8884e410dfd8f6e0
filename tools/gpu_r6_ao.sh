#!/bin/bash
# round 6 (ao): kernel-trace stats of the headline step on the final tree
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6/ao_prof
cd $R
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/ao_prof -o run -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/r6/ao_headline.log 2>&1
rc=$?; echo rc=$rc; grep '"metric"' gpurun_out/r6/ao_headline.log | cut -c1-200
find gpurun_out/r6/ao_prof -name "*kernel_stats.csv" | head -3
