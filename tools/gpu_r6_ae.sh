#!/bin/bash
# round 6 (ae): packed-batch merging off by default - full GPU suite (-x) + smoke,
# then the transparent 70B (merge off = new default, merge 64 = old) for its cost
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 960 python -u -c "
import faulthandler, sys
f = open('$R/gpurun_out/r6/ae_fh.txt', 'w')
faulthandler.dump_traceback_later(900, exit=True, file=f)
import pytest
sys.exit(pytest.main(['tests', '-m', 'gpu', '-x', '-q', '-rfE', '--timeout', '120', '--timeout-method', 'thread', '-p', 'no:cacheprovider']))
" > gpurun_out/r6/ae_suite.log 2>&1
rc=$?; echo suite rc=$rc; tail -3 gpurun_out/r6/ae_suite.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/ae_smoke.log 2>&1 || { echo smoke failed; exit 1; }
grep -o "max_logit_err_vs_fp32.: [0-9.]*" gpurun_out/r6/ae_smoke.log
timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/ae_tm70b.log 2>&1 || { echo TM_FAIL; tail -5 gpurun_out/r6/ae_tm70b.log; exit 1; }
grep '"metric"' gpurun_out/r6/ae_tm70b.log | cut -c1-200
RT_RING_MERGE_PACKED_MB=64 timeout -k 10 600 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 5 --warmup 3 > gpurun_out/r6/ae_tm70b_merge.log 2>&1 || { echo TM_FAIL; tail -5 gpurun_out/r6/ae_tm70b_merge.log; exit 1; }
grep '"metric"' gpurun_out/r6/ae_tm70b_merge.log | cut -c1-200
