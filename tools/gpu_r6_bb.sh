#!/bin/bash
# round 6 (bb): is the packed transparent-mode mismatch capacity-induced or packing-induced?
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
for v in "RT_RING_MERGE_PACKED_MB=64 RT_DEBUG_CHECK_COPY_OWNER=1"; do
  echo "== $v" >> gpurun_out/r6/bb_diag.log
  env $v timeout -k 10 200 python -u tools/diag_managed_pack.py /tmp/diagmp 2 >> gpurun_out/r6/bb_diag.log 2>&1 || { echo "rc=$?"; break; }
done
grep -v "^run\|PLAIN" gpurun_out/r6/bb_diag.log | cut -c1-600 | head -40
