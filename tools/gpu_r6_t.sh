#!/bin/bash
# round 6 (v): the full GPU suite (with -x, as the driver runs it) + smoke on the fixed tree
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
python -u -c "
import faulthandler, sys
f = open('$R/gpurun_out/r6/v_fh.txt', 'w')
faulthandler.dump_traceback_later(600, exit=True, file=f)
import pytest
sys.exit(pytest.main(['tests', '-m', 'gpu', '-x', '-q', '-rfE', '--timeout', '120', '--timeout-method', 'thread', '-p', 'no:cacheprovider']))
" > gpurun_out/r6/v_suite.log 2>&1; echo suite rc=$?; tail -3 gpurun_out/r6/v_suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/v_smoke.log 2>&1; echo smoke=$?; grep -o "max_logit_err_vs_fp32.: [0-9.]*" gpurun_out/r6/v_smoke.log
