#!/bin/bash
# round 6 (x): repeat the packed transparent-mode run and describe differences
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 420 python -u tools/diag_managed_pack.py /tmp/diagmp 6 > gpurun_out/r6/x_diag.log 2>&1
rc=$?; echo diag rc=$rc; tail -30 gpurun_out/r6/x_diag.log
