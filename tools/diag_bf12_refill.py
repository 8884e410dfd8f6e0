#!/usr/bin/env python3
"""BF12 packed refill diagnostics: staged (SDMA -> HBM stage -> k_bf12_decode)
vs fused (kernel reads the host copy) rate of a 1 GiB read-mostly buffer, with
the ring's copy counters and the huge-page backing of the host chunks."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm._native import lib  # noqa: E402


def smaps_huge(addr: int, n: int) -> dict:
    out = {}
    cur = None
    with open("/proc/self/smaps") as f:
        for line in f:
            parts = line.split()
            if "-" in parts[0] and len(parts) > 4:
                lo, hi = (int(x, 16) for x in parts[0].split("-"))
                cur = lo < addr + n and addr < hi
                continue
            if cur and parts[0].rstrip(":") in ("Rss", "AnonHugePages", "ShmemPmdMapped", "FilePmdMapped", "KernelPageSize", "MMUPageSize"):
                k = parts[0].rstrip(":")
                out[k] = out.get(k, 0) + int(parts[1])
    return out


def rate(b, n, reps=3):
    best, ring = 0.0, None
    for _ in range(reps):
        b.evict("gpu:0")
        torch.cuda.synchronize()
        s0 = lib.stats()
        t0 = time.perf_counter()
        l = b.acquire(0, rt.READ)
        l.wait(0)
        dt = time.perf_counter() - t0
        l.release()
        s1 = lib.stats()
        g = n / dt / 1e9
        if g > best:
            best = g
            ring = {k: s1[k] - s0[k] for k in ("ring_copy_ns", "ring_copy_calls", "ring_idle_ns")}
    return round(best, 1), ring


rt.init("hip", host_budget_mb=16384, hbm_budget={0: 2 << 30}, pack_host_copies=0)
lib.init_device(0, 3 << 30)
n = 1 << 30
data = (torch.randn(n // 2, device="cuda") * 0.02).to(torch.bfloat16)
b = rt.malloc_managed(n, "pk", packed_bf16=True)
b.write(data)
b.set_read_mostly(True)
host = [e for e in b.residency(0)["resident_on"] if e["tier"] == "host"][0]
base = lib.arena_stats(1, host["id"])["base"]
print("host arena", lib.arena_stats(1, host["id"]), "chunk", host["chunk"], flush=True)
print("smaps (kB) of the first 64 MB of the copy:", smaps_huge(base + host["chunk"] * (2 << 20), 64 << 20), flush=True)
for tag, cfg in (("staged", dict(bf12_stage=1)), ("staged_1eng", dict(bf12_stage=1, ans_stage_engines=1)),
                 ("fused", dict(bf12_stage=0)), ("staged_again", dict(bf12_stage=1, ans_stage_engines=15))):
    rt.configure(**cfg)
    e0 = lib.engine_bytes(0)
    r = rate(b, n)
    e1 = lib.engine_bytes(0)
    print(tag, r, "engine MB:", {i: (e1[i] - e0[i]) >> 20 for i in range(len(e1)) if e1[i] != e0[i]}, flush=True)
