#!/usr/bin/env python3
"""Host-side profile (cProfile) of the stock-torch Llama decode under
ogkm.managed() - where the dispatch thread's time goes per step (op holds with
their stable-VA remaps and copies, prefetches, aten dispatch).
    python tools/prof_torch_managed.py --model llama3-8b --steps 2"""
from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--oversub", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--context", type=int, default=1024)
    a = ap.parse_args()
    import torch

    import ogkm
    from ogkm import allocator, rt
    from ogkm._native import lib
    from ogkm.models import llama, torch_llama

    cfg = llama.CONFIGS[a.model]
    foot = torch_llama.footprint_bytes(cfg, a.batch, a.context)
    allocator.enable(managed_min_mb=1)
    rt.init("hip", hbm_budget={0: int(foot / a.oversub)}, host_budget_mb=0)
    torch.cuda.set_device(0)
    prefill = a.context - (a.warmup + a.steps) - 1
    mode = ogkm.managed()
    with mode:
        model = torch_llama.build_on_device(cfg, a.batch, a.context, "cuda", seed=1234, prefill=prefill)
        for p in model.parameters():
            if allocator.is_managed(p):
                allocator.set_read_mostly(p)
        tok = torch.randint(0, cfg.vocab, (a.batch,), device="cuda")
        pos = prefill
        for _ in range(a.warmup):
            tok = model.step(tok, pos)
            pos += 1
        torch.cuda.synchronize()
        lib.reset_counters()
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        for _ in range(a.steps):
            tok = model.step(tok, pos)
            pos += 1
        h = time.perf_counter()
        torch.cuda.synchronize()
        pr.disable()
        t1 = time.perf_counter()
    s = lib.stats()
    print(f"host enqueue {1e3 * (h - t0) / a.steps:.1f} ms/step, synchronized {1e3 * (t1 - t0) / a.steps:.1f} "
          f"ms/step; vmm_remaps/step {s['vmm_remaps'] / a.steps:.0f} tlb_flushes/step {s['tlb_flushes'] / a.steps:.1f} "
          f"htd GB/step {s['bytes_xfer_htd'] / a.steps / 1e9:.2f}", flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
