#!/bin/bash
# round 6 (au): stable_batch_blocks 32 (default) vs 128 vs 256 on one box, correctness at 128
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
RT_STABLE_BATCH_BLOCKS=128 timeout -k 10 300 python -u tools/diag_managed_pack.py /tmp/diagmp 4 > gpurun_out/r6/au_diag.log 2>&1 || { echo "diag rc=$?"; exit 1; }
grep DIAG_DONE gpurun_out/r6/au_diag.log
for v in 32 128 256 32 128; do
  RT_STABLE_BATCH_BLOCKS=$v timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/au_tm70b.log 2>&1 || { echo TM_FAIL; tail -5 gpurun_out/r6/au_tm70b.log; exit 1; }
  echo "$v $(grep '"metric"' gpurun_out/r6/au_tm70b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["aux"]["host_ms_per_step"])')" | tee -a gpurun_out/r6/au_tm70b_ab.txt
done
