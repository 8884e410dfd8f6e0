#!/bin/bash
ulimit -c 0
mkdir -p gpurun_out/r3
for cfg in "256 1024 2" "64 256 4" "16 64 8"; do
  set -- $cfg
  timeout -k 10 150 python tools/bench_managed.py --tensors 8 --mb $1 --arena-mb $2 --iters $3 --mode dispatch > gpurun_out/r3/bm_d$1.log 2>&1 || exit $?
  tail -1 gpurun_out/r3/bm_d$1.log
done
timeout -k 10 150 python tools/bench_managed.py --tensors 8 --mb 256 --arena-mb 1024 --iters 2 --mode park > gpurun_out/r3/bm_p256.log 2>&1 || exit $?
tail -1 gpurun_out/r3/bm_p256.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_managed_mode_gpu.py > gpurun_out/r3/mode_test.log 2>&1; echo mode_test rc=$?; tail -2 gpurun_out/r3/mode_test.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --marker-trace --memory-copy-trace --stats --output-format csv -d /root/repo/gpurun_out/r3/prof_disp -o run -- python3 /root/repo/tools/bench_managed.py --tensors 8 --mb 256 --arena-mb 1024 --iters 2 --mode dispatch --trace-level 2 > /root/repo/gpurun_out/r3/prof_disp.log 2>&1
echo prof rc=$?
