#!/bin/bash
# Round 5 (aa): transparent 70B block census - which blocks refills move raw.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
OGKM_TM_CENSUS=1 OGKM_PACK=1 timeout -k 10 700 python -u bench.py --torch-managed --model llama3-70b --oversub 2 --steps 3 --warmup 3 > gpurun_out/r5/aa_tm_census.log 2>&1 || { echo TM_FAIL; tail -30 gpurun_out/r5/aa_tm_census.log; exit 1; }
grep '^{' gpurun_out/r5/aa_tm_census.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step']); print(json.dumps(a['block_census'], indent=1)); print(a['pack'])"
echo ALL_OK
