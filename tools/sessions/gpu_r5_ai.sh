#!/bin/bash
# Round 5 (ai): the default bench with the new step defaults; PMC counters of the
# tp8-shape decode attention (why it is latency-bound).
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 700 python -u bench.py > gpurun_out/r5/ai_bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r5/ai_bench.log; exit 1; }
grep '^{' gpurun_out/r5/ai_bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['steps'], d['warmup'])"
cd /tmp
for shape in 70b-tp8 70b; do
  SHAPE=$shape ITERS=20 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD FETCH_SIZE -d $R/gpurun_out/r5/ai_pmc_$shape -o pmc -- python3 $R/tools/bench_attn.py > $R/gpurun_out/r5/ai_pmc_$shape.log 2>&1 || { echo PMC_FAIL $shape; tail -20 $R/gpurun_out/r5/ai_pmc_$shape.log; exit 1; }
  echo "pmc $shape done"
done
echo ALL_OK
