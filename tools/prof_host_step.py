#!/usr/bin/env python3
"""Host-side cost of one TieredLlama decode step (cProfile), e.g. the 70B tp8
rank-0 shard simulated on one GPU, where the host enqueue time is close to the
step time. Prints the top functions by own time.
    python tools/prof_host_step.py --model llama3-70b --simulate-tp 8"""
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
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--simulate-tp", type=int, default=8)
    ap.add_argument("--oversub", type=float, default=2.0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--weight-format", default="ans")
    ap.add_argument("--kv-format", default="ans")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--planner", default="static")
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    import torch

    from ogkm import rt
    from ogkm.models import llama
    rt.init("hip", host_budget_mb=0)
    cfg = llama.CONFIGS[a.model]
    m = llama.TieredLlama(cfg, batch=a.batch, context=1024, max_new_tokens=2 * a.steps + a.warmup + 8, oversub=a.oversub,
                          tp_rank=0, tp_world=a.simulate_tp, weight_format=a.weight_format, kv_format=a.kv_format,
                          lookahead=1, planner=a.planner)
    tok = torch.zeros(a.batch, dtype=torch.int64, device="cuda")
    for _ in range(a.warmup):
        tok = m.step(tok)
    torch.cuda.synchronize()
    # unprofiled: host enqueue time vs synchronized step time (GPU-starved when close)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tok = m.step(tok)
    h = time.perf_counter() - t0
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"host enqueue {1e3 * h / a.steps:.2f} ms/step (unprofiled), synchronized {1e3 * t / a.steps:.2f} ms/step")
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        tok = m.step(tok)
    pr.disable()
    h = time.perf_counter() - t0
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"host enqueue {1e3 * h / a.steps:.1f} ms/step (profiled), synchronized {1e3 * t / a.steps:.1f} ms/step")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    m.close()


if __name__ == "__main__":
    main()
