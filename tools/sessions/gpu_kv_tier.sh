# KV tiering on the GPU: model tests, then the long-context line
# (Llama-3-70B, ctx 32k, batch 8: the bf16 KV cache alone is 86 GB).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_gpu_runtime.py -x -v --timeout 200 --timeout-method thread -k "kv_tiering or fragmented" > gpurun_out/gpu_kvtier.log 2>&1; rc=$?
tail -4 gpurun_out/gpu_kvtier.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench.py --context 32768 --batch 8 --kv-format bf16 --kv-tiering --steps 3 --warmup 1 --no-aux --verbose > gpurun_out/bench_longctx.log 2>&1 || { echo LONGCTX_FAIL; tail -20 gpurun_out/bench_longctx.log; exit 1; }
grep '^{' gpurun_out/bench_longctx.log | cut -c1-900
