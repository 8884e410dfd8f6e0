# 70B 2x variants on one GPU: planner off (runtime LRU residency) and the
# codec-free comparator (raw bf16 weights + KV, no packed host copies).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --steps 3 --warmup 1 --no-aux --planner off > gpurun_out/bench_planner_off.log 2>&1 || { echo PLANNER_OFF_FAIL; tail -20 gpurun_out/bench_planner_off.log; exit 1; }
grep '^{' gpurun_out/bench_planner_off.log | cut -c1-400
timeout -k 10 500 python bench.py --steps 3 --warmup 1 --no-aux --weights bf16 --kv-format bf16 --no-packed > gpurun_out/bench_codec_free.log 2>&1 || { echo CODEC_FREE_FAIL; tail -20 gpurun_out/bench_codec_free.log; exit 1; }
grep '^{' gpurun_out/bench_codec_free.log | cut -c1-400
