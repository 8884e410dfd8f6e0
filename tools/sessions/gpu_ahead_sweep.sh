# Host run-ahead bound sweep on the 70B 2x headline (GPU-side lease waits).
set -o pipefail
mkdir -p gpurun_out
for k in 0 1 3 6; do
  OGKM_MAX_AHEAD=$k timeout -k 10 420 python bench.py --steps 5 --warmup 2 --no-aux > gpurun_out/ahead_$k.log 2>&1 || { echo "ahead $k FAILED"; tail -5 gpurun_out/ahead_$k.log; exit 1; }
  echo "max_ahead=$k $(grep '^{' gpurun_out/ahead_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["aux"]["link_gbps_per_gpu"])')"
done
