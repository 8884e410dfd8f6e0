#!/bin/bash
# round 6 (aa): the merged-batch ordering fix - packed transparent-mode repeats,
# then the full GPU suite (-x, as the driver runs it) and smoke
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 300 python -u tools/diag_managed_pack.py /tmp/diagmp 4 > gpurun_out/r6/aa_diag.log 2>&1
rc=$?; echo diag rc=$rc; grep -v "^run" gpurun_out/r6/aa_diag.log | cut -c1-250
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 960 python -u -c "
import faulthandler, sys
f = open('$R/gpurun_out/r6/aa_fh.txt', 'w')
faulthandler.dump_traceback_later(900, exit=True, file=f)
import pytest
sys.exit(pytest.main(['tests', '-m', 'gpu', '-x', '-q', '-rfE', '--timeout', '120', '--timeout-method', 'thread', '-p', 'no:cacheprovider']))
" > gpurun_out/r6/aa_suite.log 2>&1
rc=$?; echo suite rc=$rc; tail -3 gpurun_out/r6/aa_suite.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/aa_smoke.log 2>&1; echo smoke=$?; grep -o "max_logit_err_vs_fp32.: [0-9.]*" gpurun_out/r6/aa_smoke.log
