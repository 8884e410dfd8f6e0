#!/usr/bin/env python3
"""Streaming microbenchmark: host tier -> HBM through the runtime (acquire after
evict), raw bf16 vs BF12-packed host copies, across copy / decode workgroup
counts. Prints one JSON line per configuration (GB/s of bf16 delivered and GB/s
on the link)."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm._native import lib  # noqa: E402


def run(nbytes: int, packed: bool, iters: int = 3) -> dict:
    b = rt.malloc_managed(nbytes, "s", packed_bf16=packed)
    b.write((torch.randn(nbytes // 2, device="cuda") * 0.02).to(torch.bfloat16))
    b.set_read_mostly(True)
    times = []
    for _ in range(iters + 1):
        b.evict("gpu:0")
        torch.cuda.synchronize()
        lib.reset_counters()
        t0 = time.perf_counter()
        l = b.acquire(0, rt.READ)
        l.wait(0)
        times.append(time.perf_counter() - t0)
        l.release()
    s = lib.stats()
    dt = min(times[1:])
    b.free()
    link = s["bytes_xfer_htd"]
    return {"packed": packed, "delivered_gbps": round(nbytes / dt / 1e9, 2), "link_gbps": round(link / dt / 1e9, 2)}


def main() -> None:
    rt.init("hip", hbm_budget={0: 4 << 30})
    n = 1 << 30
    for wg in (32, 64, 128):
        lib.configure("copy_workgroups", wg)
        print(json.dumps({"copy_workgroups": wg, **run(n, False)}), flush=True)
    lib.configure("copy_workgroups", 64)
    for wg in (128, 256, 512):
        lib.configure("decode_workgroups", wg)
        print(json.dumps({"decode_workgroups": wg, **run(n, True)}), flush=True)
    lib.shutdown()


if __name__ == "__main__":
    main()
