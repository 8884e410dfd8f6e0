#!/bin/bash
# round 6: segmented packing + allocator GPU tests, config-2 allocator A/B
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_packing_gpu.py tests/test_gpu_runtime.py -q -k "packing or segmented or packed or allocator or bf12" --timeout 120 --timeout-method thread > gpurun_out/r6/e_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r6/e_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r6/e_c2_caching_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/r6/e_c2_caching_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('caching', d['value'], d['ms_per_step'])"
  timeout -k 10 400 python -u bench.py --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --allocator > gpurun_out/r6/e_c2_alloc_$i.log 2>&1 || { tail -5 gpurun_out/r6/e_c2_alloc_$i.log; exit 1; }
  grep '^{' gpurun_out/r6/e_c2_alloc_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('arena', d['value'], d['ms_per_step'], d['config'].get('torch_allocator'))"
done
