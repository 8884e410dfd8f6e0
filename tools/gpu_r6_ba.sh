#!/bin/bash
# round 6 (ba): is the packed transparent-mode mismatch capacity-induced or packing-induced?
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
for v in "RT_RING_MERGE_PACKED_MB=64 OGKM_DIAG_STABLE=1 OGKM_DIAG_SNAP=layers.15.linear1.weight OGKM_DIAG_SECOND_OUT=/tmp/sc.pt"; do
  echo "== $v" >> gpurun_out/r6/ba_diag.log
  env $v timeout -k 10 200 python -u tools/diag_managed_pack.py /tmp/diagmp 3 >> gpurun_out/r6/ba_diag.log 2>&1 || { echo "rc=$?"; break; }
done
grep -v "^run\|PLAIN" gpurun_out/r6/ba_diag.log | cut -c1-250; grep "^run" gpurun_out/r6/ba_diag.log | cut -c1-60
