#!/bin/bash
# round 6 (n): kernel traces of the BF12 refill diagnostic, old tree vs new
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R/old_tree && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/r6/n_old -o old -- python3 diag_bf12_refill.py > $R/gpurun_out/r6/n_old.log 2>&1 || { echo OLD_FAIL; tail -5 $R/gpurun_out/r6/n_old.log; exit 1; }
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/r6/n_new -o new -- python3 tools/diag_bf12_refill.py > $R/gpurun_out/r6/n_new.log 2>&1 || { echo NEW_FAIL; tail -5 $R/gpurun_out/r6/n_new.log; exit 1; }
grep -h "staged\|fused" $R/gpurun_out/r6/n_old.log $R/gpurun_out/r6/n_new.log | cut -c1-120
for f in $(find $R/gpurun_out/r6/n_old $R/gpurun_out/r6/n_new -name "*kernel_stats.csv"); do echo "== $f"; head -8 $f | cut -c1-200; done
echo ALL_OK
