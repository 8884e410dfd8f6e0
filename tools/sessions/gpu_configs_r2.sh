# Round-2 final build: refresh the non-headline configuration lines.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/configs_r2.log
run() {
  echo "== $*" >> gpurun_out/configs_r2.log
  timeout -k 10 600 "$@" >> gpurun_out/configs_r2.log 2>&1 || { echo "FAIL $*"; tail -8 gpurun_out/configs_r2.log; exit 1; }
  grep '^{' gpurun_out/configs_r2.log | tail -1 | cut -c1-260
}
run python bench.py --model llama3-70b --simulate-tp 8 --steps 4 --warmup 1 --no-aux
run python bench.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 3 --warmup 1 --no-aux
run python bench.py --tiers host+cxl --steps 3 --warmup 1 --no-aux
run python bench.py --model llama3-8b --oversub 1.0 --allocator --steps 10 --warmup 3 --no-aux
run python bench.py --context 32768 --batch 8 --kv-format bf16 --kv-tiering --steps 3 --warmup 1 --no-aux
