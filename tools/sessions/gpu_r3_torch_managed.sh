#!/bin/bash
ulimit -c 0
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u bench.py --torch-managed --model llama3-8b --oversub 2 --steps 4 --warmup 3 > gpurun_out/r3/tm8b.log 2>&1
echo rc=$?
grep -v "^W20\|amdgpu.ids" gpurun_out/r3/tm8b.log | tail -5
