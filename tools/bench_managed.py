"""Managed torch tensors: park/unpark (or transparent dispatch-mode) round-trip
bandwidth when the tensors oversubscribe the HBM arena.

N tensors of S MB live in an arena of A MB; the loop touches them cyclically
(each touch: make resident -> x.add_(1) -> evictable again), so every touch
brings S MB in over PCIe and pushes S MB of another tensor out. Reports the
touched bytes per second ("round trip GB/s") plus runtime counter deltas.

    python tools/bench_managed.py --tensors 8 --mb 256 --arena-mb 1024 --iters 3
    python tools/bench_managed.py --mode dispatch ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tensors", type=int, default=8)
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--arena-mb", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--mode", choices=["park", "dispatch"], default="park")
    ap.add_argument("--sync-phases", action="store_true", help="synchronize after each phase (per-phase times)")
    ap.add_argument("--lazy-unmap", action="store_true")
    ap.add_argument("--batch-blocks", type=int, default=32)
    ap.add_argument("--trace-level", type=int, default=1)
    a = ap.parse_args()

    import torch
    import ogkm  # noqa: F401
    from ogkm import allocator, rt

    allocator.enable(managed_min_mb=4)
    rt.init("hip", hbm_budget={0: a.arena_mb << 20}, stable_lazy_unmap=int(a.lazy_unmap),
            stable_batch_blocks=a.batch_blocks, perf_workingset_active_pct=0, trace_ranges=a.trace_level)
    n = a.mb << 20
    xs = []
    for i in range(a.tensors):
        x = torch.full((n // 4,), float(i), device="cuda")
        allocator.park(x)
        xs.append(x)
    torch.cuda.synchronize()

    mode = None
    if a.mode == "dispatch":
        mode = ogkm.managed(lookahead_bytes=0)
        mode.__enter__()

    def touch(x):
        if a.mode == "park":
            allocator.unpark(x)
            x.add_(1.0)
            allocator.park(x)
        else:
            x.add_(1.0)

    # warm-up lap (first host registrations, first evictions)
    for x in xs:
        touch(x)
    torch.cuda.synchronize()
    s0 = rt.stats()
    t0 = time.perf_counter()
    phase = {"touch": 0.0}
    for _ in range(a.iters):
        for x in xs:
            t1 = time.perf_counter()
            touch(x)
            if a.sync_phases:
                torch.cuda.synchronize()
            phase["touch"] += time.perf_counter() - t1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s1 = rt.stats()
    if mode is not None:
        mode.__exit__(None, None, None)
    htd = s1.get("bytes_xfer_htd", 0) - s0.get("bytes_xfer_htd", 0)
    touched = a.iters * a.tensors * n
    keys = ["bytes_xfer_htd", "bytes_xfer_dth", "evictions", "vmm_remaps", "tlb_flushes", "ring_submissions",
            "alloc_retries"]
    delta = {k: s1.get(k, 0) - s0.get(k, 0) for k in keys if k in s1}
    # correctness: every tensor was touched iters+1 times
    ok = True
    for i, x in enumerate(xs):
        allocator.unpark(x)
        v = float(x[:: max(1, x.numel() // 64)].min()), float(x[:: max(1, x.numel() // 64)].max())
        allocator.park(x)
        ok &= v == (i + a.iters + 1.0, i + a.iters + 1.0)
    print(json.dumps({"mode": a.mode, "tensors": a.tensors, "mb": a.mb, "arena_mb": a.arena_mb, "iters": a.iters,
                      "seconds": round(dt, 4), "round_trip_gbps": round(touched / dt / 1e9, 2),
                      "htd_gbps": round(htd / dt / 1e9, 2),
                      "ms_per_touch": round(dt / (a.iters * a.tensors) * 1e3, 3), "correct": ok, "counters": delta}))


if __name__ == "__main__":
    main()
