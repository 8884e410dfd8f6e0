# Sweep migration-engine knobs on the 70B 2x-oversubscribed decode bench.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep70b.log
run() {
  echo "== $*" >> gpurun_out/sweep70b.log
  env "$@" timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-aux ${BENCH_ARGS} >> gpurun_out/sweep70b.log 2>&1 || { echo "FAIL $*"; tail -5 gpurun_out/sweep70b.log; exit 1; }
  grep '^{' gpurun_out/sweep70b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'], d['aux']['link_gbps_per_gpu'])"
}
for cfg in ${SWEEP}; do run $(echo $cfg | tr '+' ' '); done
