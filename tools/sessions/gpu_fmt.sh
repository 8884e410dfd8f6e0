#!/bin/bash
# GPU tests, then one 70B bench per weight/KV format in ${FMTS} (default "bf11 ans"); each step time-limited.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; grep -E "^(FAILED|E )" gpurun_out/gpu_tests.log | head -30; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
  grep -E "HBM unpack" gpurun_out/gpu_tests.log
fi
for f in ${FMTS:-bf11 ans}; do
  timeout -k 10 450 python bench.py --steps 5 --warmup 2 --no-aux --weights $f --kv-format $f ${BENCH_ARGS} > gpurun_out/bench_$f.log 2>&1 || { echo BENCH_FAIL $f; tail -30 gpurun_out/bench_$f.log; exit 1; }
  grep '^{' gpurun_out/bench_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$f', d['value'], 'tok/s', d['ms_per_step'], 'ms', c['streamed_gb_per_step_per_gpu'], 'GB/step', c['resident_layers'], 'res', d['aux']['link_gbps_per_gpu'], 'GB/s')"
done
