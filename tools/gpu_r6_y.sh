#!/bin/bash
# round 6 (y): A/B of the packed transparent-mode mismatch over allocator knobs
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
for v in "RT_TORCH_ALLOC_EMPTY_SLABS=0" "RT_TORCH_ALLOC_CACHE_MB=0" "RT_TORCH_ALLOC_EMPTY_SLABS=0 RT_TORCH_ALLOC_CACHE_MB=0"; do
  echo "== $v" >> gpurun_out/r6/y_diag.log
  env $v timeout -k 10 200 python -u tools/diag_managed_pack.py /tmp/diagmp 2 >> gpurun_out/r6/y_diag.log 2>&1 || { echo "rc=$?"; break; }
done
grep -v "^run\|PLAIN" gpurun_out/r6/y_diag.log | cut -c1-250; grep -c "^run" gpurun_out/r6/y_diag.log
