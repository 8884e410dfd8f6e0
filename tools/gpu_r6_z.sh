#!/bin/bash
# round 6 (z): is the packed transparent-mode mismatch capacity-induced or packing-induced?
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
for v in "RT_TORCH_ALLOC_EMPTY_SLABS=0 OGKM_TEST_ARENA_MB=336" "RT_TORCH_ALLOC_EMPTY_SLABS=0 OGKM_TEST_ARENA_MB=352" "RT_PACK_HOST_COPIES=0" "RT_ANS_STAGE_MB=0"; do
  echo "== $v" >> gpurun_out/r6/z_diag.log
  env $v timeout -k 10 200 python -u tools/diag_managed_pack.py /tmp/diagmp 2 >> gpurun_out/r6/z_diag.log 2>&1 || { echo "rc=$?"; break; }
done
grep -v "^run\|PLAIN" gpurun_out/r6/z_diag.log | cut -c1-250; grep "^run" gpurun_out/r6/z_diag.log | cut -c1-60
