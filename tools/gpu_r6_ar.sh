#!/bin/bash
# round 6 (ar): final tree - full GPU suite (-x), smoke, headline bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 960 python -u -c "
import faulthandler, sys
f = open('$R/gpurun_out/r6/ar_fh.txt', 'w')
faulthandler.dump_traceback_later(900, exit=True, file=f)
import pytest
sys.exit(pytest.main(['tests', '-m', 'gpu', '-x', '-q', '-rfE', '--timeout', '120', '--timeout-method', 'thread', '-p', 'no:cacheprovider']))
" > gpurun_out/r6/ar_suite.log 2>&1
rc=$?; echo suite rc=$rc; tail -2 gpurun_out/r6/ar_suite.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/ar_smoke.log 2>&1 || { echo smoke failed; exit 1; }
grep -o "max_logit_err_vs_fp32.: [0-9.]*" gpurun_out/r6/ar_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r6/ar_headline.log 2>&1 || { echo HEAD_FAIL; tail -5 gpurun_out/r6/ar_headline.log; exit 1; }
grep '"metric"' gpurun_out/r6/ar_headline.log | cut -c1-200
