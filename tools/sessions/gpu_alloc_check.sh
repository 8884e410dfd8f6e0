# Pluggable allocator on the GPU: stream-ordered frees test + the config-2 bench
# (Llama-3-8B, HBM only, torch tensors in the runtime's arena).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread -k "allocator" > gpurun_out/gpu_alloc.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_alloc.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --model llama3-8b --oversub 1.0 --steps 10 --warmup 3 --no-aux --allocator > gpurun_out/bench8b_alloc.log 2>&1 || { echo B8_FAIL; tail -20 gpurun_out/bench8b_alloc.log; exit 1; }
grep '^{' gpurun_out/bench8b_alloc.log | cut -c1-600
timeout -k 10 400 python bench.py --model llama3-8b --oversub 1.0 --steps 10 --warmup 3 --no-aux > gpurun_out/bench8b.log 2>&1 || { echo B8N_FAIL; tail -20 gpurun_out/bench8b.log; exit 1; }
grep '^{' gpurun_out/bench8b.log | cut -c1-300
