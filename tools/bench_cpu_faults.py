#!/usr/bin/env python3
"""North-star config 1: CPU-fault simulation over 1 GB of synthetic managed
memory on the CPU-only (fake) backend.

The range is written, moved to the fake GPU (its CPU view loses every
mapping), then read back through the CPU view by torch's CPU kernels with
`--threads` threads: every first touch of a page is a real SIGSEGV, posted by
the async-signal-safe handler to the CPU-fault service thread
(csrc/core/cpu_fault.cpp), serviced (migration GPU -> host + remap) and
replayed. Two passes:

  * prefetch off: one fault per 4 KiB page -> faults/s (service latency bound);
  * prefetch on (default policy, uvm_perf_prefetch 51% tree): the block-level
    prefetch turns most first touches into 2 MB migrations -> GB/s.

Prints one JSON line per pass. The reference's equivalent is the UVM CPU fault
path (uvm.c:576 -> uvm_va_space_cpu_fault, uvm_va_space.c:2482-2590).

    python tools/bench_cpu_faults.py [--gb 1] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm._native import lib  # noqa: E402


def one_pass(size: int, prefetch: bool, threads: int) -> dict:
    lib.configure("perf_prefetch_enable", 1 if prefetch else 0)
    b = rt.malloc_managed(size, "cf-bench")
    n = size // 4
    src = torch.arange(n, dtype=torch.int32)
    b.write(src)
    b.migrate("gpu:0")                         # the CPU view is now unmapped
    assert all(r["tier"] == "gpu" for r in b.residency(0)["resident_on"])
    lib.reset_counters()
    s0 = lib.stats()["cpu_faults_serviced"]
    v = b.cpu_view(torch.int32)
    torch.set_num_threads(threads)
    t0 = time.perf_counter()
    total = int(v.sum(dtype=torch.int64))      # touches every page of the view
    dt = time.perf_counter() - t0
    st = lib.stats()
    faults = st["cpu_faults_serviced"] - s0
    assert total == n * (n - 1) // 2, "data mismatch after CPU faults"
    b.free()
    return {
        "metric": f"CPU-fault read of {size >> 30} GB managed memory ({'prefetch on' if prefetch else 'prefetch off'})",
        "value": round(size / dt / 1e9, 3), "unit": "GB/s", "higher_is_better": True,
        "faults": faults, "faults_per_s": round(faults / dt, 1), "seconds": round(dt, 3),
        "migrated_bytes_dth": st["bytes_xfer_dth"], "threads": threads,
        "config": {"backend": "fake (CPU-only)", "data": "synthetic int32 ramp", "north_star": "config 1"},
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.0)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    size = int(a.gb * (1 << 30))
    rt.init("fake", fake_devices=1, fake_hbm_mb=int(a.gb * 1024) + 256, host_budget_mb=int(a.gb * 1024) * 3 + 512)
    lib.init_device(0, size + (64 << 20))
    for prefetch in (False, True):
        print(json.dumps(one_pass(size, prefetch, a.threads)), flush=True)
    lib.shutdown()


if __name__ == "__main__":
    main()
