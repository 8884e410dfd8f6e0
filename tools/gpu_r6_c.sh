#!/bin/bash
# round 6: smoke + config-2 allocator A/B (torch caching vs ogkm arena), same box
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/c_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r6/c_smoke.log; exit 1; }
tail -2 gpurun_out/r6/c_smoke.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 > gpurun_out/r6/c_c2_caching_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/r6/c_c2_caching_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('caching', d['value'], d['ms_per_step'])"
  timeout -k 10 400 python -u bench.py --model llama3-8b --oversub 1.0 --steps 30 --warmup 5 --allocator > gpurun_out/r6/c_c2_alloc_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/r6/c_c2_alloc_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('arena', d['value'], d['ms_per_step'], d['config'].get('torch_allocator'))"
done
