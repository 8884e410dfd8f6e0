#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/probe_vmm_remap.py sync 2>&1 | grep -v amdgpu.ids | tail -3
for i in 1 2; do timeout -k 10 120 python -u tools/debug_managed_alloc.py > gpurun_out/dbg_managed_$i.log 2>&1; grep -E "^stats|tensor|DUP|Error" gpurun_out/dbg_managed_$i.log | head -8; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -k "managed or allocator or stable" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/managed_tests.log 2>&1; echo tests rc=$?
grep -E "MANAGED_OK|passed|failed" gpurun_out/managed_tests.log | cut -c1-300
