#!/bin/bash
# Round-3 GPU session: transparent managed mode + stable-VA placement.
# Each GPU step has its own time limit; a crash / abort / timeout ends the
# session (rc other than 0 or 1), an ordinary test failure (rc 1) does not.
ulimit -c 0
mkdir -p gpurun_out/r3
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  tail -3 "gpurun_out/r3/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step mode_test 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_managed_mode_gpu.py
step health 200 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "health"
step bm_dispatch 150 python tools/bench_managed.py --tensors 8 --mb 256 --arena-mb 1024 --iters 2 --mode dispatch
step bm_dispatch64 150 python tools/bench_managed.py --tensors 8 --mb 64 --arena-mb 256 --iters 4 --mode dispatch
grep -h "MANAGED_OK\|device_health" gpurun_out/r3/mode_test.log gpurun_out/r3/health.log | head -5
for f in bm_dispatch bm_dispatch64; do tail -1 gpurun_out/r3/$f.log; done
