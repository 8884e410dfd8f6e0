#!/usr/bin/env python3
"""Managed-allocator oversubscription check with per-block diagnostics: 8 x 64 MB
torch tensors on a 256 MB arena, park / unpark each in turn; on a mismatch,
print which 2 MB blocks are wrong, what value they hold (= which tensor's data)
and their residency."""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import allocator, rt  # noqa: E402
from ogkm._native import lib  # noqa: E402

allocator.enable(managed_min_mb=4)
rt.init("hip", hbm_budget={0: 256 << 20})
N = 16 << 20
xs = []
for i in range(8):
    x = torch.full((N,), float(i), device="cuda")
    allocator.park(x)
    xs.append(x)
torch.cuda.synchronize()
ids = {}
for rid in lib.range_ids():
    info = lib.range_info(rid)
    if info["name"] == "torch":
        ids[info["dev_va"]] = rid


def dup_check(tag):
    """HBM chunks claimed by two blocks of torch ranges (must never happen)."""
    owners = {}
    for rid in lib.range_ids():
        info = lib.range_info(rid)
        if info["name"] != "torch":
            continue
        for blk in range(0, info["size"], 2 << 20):
            for r in lib.residency_info(rid, blk)["resident_on"]:
                if r["tier"] == "gpu":
                    owners.setdefault(r["chunk"], []).append((rid, blk >> 21))
    d = {c: o for c, o in owners.items() if len(o) > 1}
    if d:
        print(f"  DUP after {tag}: {dict(list(d.items())[:4])} arena_check {lib.arena_check(0, 0)!r}", flush=True)
    return len(d)


bad_total = 0
dup_check("fill")
t0 = time.perf_counter()
for i, x in enumerate(xs):
    allocator.unpark(x)
    torch.cuda.synchronize()
    dup_check(f"unpark {i}")
    blk = x.view(32, -1)
    eq = blk == float(i)
    dup_check(f"eq {i}")
    ok = eq.all(dim=1).cpu()
    del eq
    if not bool(ok.all()):
        bad = [j for j in range(32) if not bool(ok[j])]
        bad_total += len(bad)
        rid = ids.get(x.data_ptr())
        print(f"tensor {i}: {len(bad)} bad blocks {bad[:8]}", flush=True)
        for j in bad[:4]:
            vals = torch.unique(blk[j]).cpu().tolist()[:6]
            res = lib.residency_info(rid, j << 21) if rid else {}
            print(f"   block {j}: values {vals} residency {res.get('resident_on')} mapped {res.get('mapped_on')}",
                  flush=True)
    y = x * 2
    torch.cuda.synchronize()
    dup_check(f"y {i}")
    del y
    allocator.park(x)
torch.cuda.synchronize()
print("stats", allocator.managed_stats(0), {k: lib.stats()[k] for k in ("evictions", "thrashing_detected")},
      "bad blocks", bad_total, "time", round(time.perf_counter() - t0, 3), flush=True)
