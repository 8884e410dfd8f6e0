#!/bin/bash
# round 6 (at): larger stable-VA placement groups instead of worker-side batch merging
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
for v in 64 128; do
  echo "== stable_batch_blocks $v" >> gpurun_out/r6/at_diag.log
  RT_STABLE_BATCH_BLOCKS=$v timeout -k 10 200 python -u tools/diag_managed_pack.py /tmp/diagmp 2 >> gpurun_out/r6/at_diag.log 2>&1 || { echo "diag rc=$?"; exit 1; }
  RT_STABLE_BATCH_BLOCKS=$v timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/at_tm70b_$v.log 2>&1 || { echo TM_FAIL; tail -5 gpurun_out/r6/at_tm70b_$v.log; exit 1; }
  grep '"metric"' gpurun_out/r6/at_tm70b_$v.log | cut -c1-170
done
grep "DIAG_DONE\|==" gpurun_out/r6/at_diag.log
