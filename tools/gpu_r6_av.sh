#!/bin/bash
# round 6 (av): transparent 70B, packed-batch merging off (default) vs on, alternating on one box
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
for v in 0 64 0 64; do
  RT_RING_MERGE_PACKED_MB=$v timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/av_tm70b.log 2>&1 || { echo TM_FAIL; tail -5 gpurun_out/r6/av_tm70b.log; exit 1; }
  echo "merge_mb=$v $(grep '"metric"' gpurun_out/r6/av_tm70b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["aux"]["ring_per_step"])')" | tee -a gpurun_out/r6/av_tm70b_ab.txt
done
