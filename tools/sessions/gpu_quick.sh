# Floor (all resident) + headline bench, each time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-aux --oversub 1.0 > gpurun_out/floor.log 2>&1 || { echo FLOOR_FAIL; tail -20 gpurun_out/floor.log; exit 1; }
grep '^{' gpurun_out/floor.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('floor', d['value'], d['ms_per_step'])"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench70b.log 2>&1 || { echo B70_FAIL; tail -30 gpurun_out/bench70b.log; exit 1; }
grep '^{' gpurun_out/bench70b.log
