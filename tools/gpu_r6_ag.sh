#!/bin/bash
# round 6 (ag): headline bench on the final tree (merge off = default) and with merging on
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 500 python -u bench.py > gpurun_out/r6/ag_headline.log 2>&1 || { echo HEAD_FAIL; tail -5 gpurun_out/r6/ag_headline.log; exit 1; }
grep '"metric"' gpurun_out/r6/ag_headline.log | cut -c1-260
RT_RING_MERGE_PACKED_MB=64 timeout -k 10 500 python -u bench.py > gpurun_out/r6/ag_headline_merge.log 2>&1 || { echo HEAD_FAIL; tail -5 gpurun_out/r6/ag_headline_merge.log; exit 1; }
grep '"metric"' gpurun_out/r6/ag_headline_merge.log | cut -c1-260
