#!/bin/bash
# Round 5 (y): transparent 70B with the new staging defaults (4 engines, 128 MB, 64 MB merges)
# vs 8 engines vs the old defaults; kernel traces of the default (planner off) 70B headline step and of
# config 2 (8B HBM-resident, runtime-decided residency), timed steps only.
set -o pipefail
ulimit -c 0
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
tm() {
  local tag=$1; shift
  env "$@" OGKM_PACK=1 timeout -k 10 600 python -u $R/bench.py --torch-managed --model llama3-70b --oversub 2 --steps 4 --warmup 3 > $R/gpurun_out/r5/y_tm_$tag.log 2>&1 || { echo TM_FAIL $tag; tail -30 $R/gpurun_out/r5/y_tm_$tag.log; return 1; }
  grep '^{' $R/gpurun_out/r5/y_tm_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['aux']; print('tm $tag', d['value'], d['ms_per_step'], a['htd_gb_per_step'], a['ring_per_step'], a['host_ms_per_step'])"
}
cd $R
tm defaults && tm eng_ff RT_ANS_STAGE_ENGINES=0xFF && tm old_defaults RT_ANS_STAGE_ENGINES=0x9 RT_ANS_STAGE_MB=64 RT_RING_MERGE_PACKED_MB=24 || exit 1
cd /tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/y_prof_70b -o run -- python3 $R/bench.py --no-aux --steps 3 --warmup 3 > $R/gpurun_out/r5/y_prof_70b.log 2>&1 || { echo PROF70_FAIL; tail -20 $R/gpurun_out/r5/y_prof_70b.log; exit 1; }
grep '^{' $R/gpurun_out/r5/y_prof_70b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('70b under profiler', d['value'], d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/y_prof_c2 -o run -- python3 $R/bench.py --no-aux --model llama3-8b --oversub 1.0 --steps 20 --warmup 5 > $R/gpurun_out/r5/y_prof_c2.log 2>&1 || { echo PROFC2_FAIL; tail -20 $R/gpurun_out/r5/y_prof_c2.log; exit 1; }
grep '^{' $R/gpurun_out/r5/y_prof_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 under profiler', d['value'], d['ms_per_step'])"
cd $R
python3 tools/rocpd_summary.py $(find gpurun_out/r5/y_prof_70b -name "*.db" | head -1) 14 --last-ms 1500
python3 tools/rocpd_summary.py $(find gpurun_out/r5/y_prof_c2 -name "*.db" | head -1) 12 --last-ms 132
echo ALL_OK
