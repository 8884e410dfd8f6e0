# North-star configs beyond the headline: 405B tp8 shard (simulated) on three tiers, 70B three-tier,
# 8B HBM-resident allocator baseline (config 2).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/configs.log
run() {
  echo "== $*" >> gpurun_out/configs.log
  timeout -k 10 420 "$@" >> gpurun_out/configs.log 2>&1 || { echo "FAIL $*"; tail -8 gpurun_out/configs.log; exit 1; }
  grep '^{' gpurun_out/configs.log | tail -1 | cut -c1-900
}
run python bench.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 3 --warmup 1 --no-aux
run python bench.py --tiers host+cxl --steps 3 --warmup 1 --no-aux
run python bench.py --model llama3-8b --oversub 1.0 --steps 5 --warmup 2 --no-aux
