#!/usr/bin/env python3
"""Per-step diagnostics of the first decode steps after load: wall time and the
runtime's transfer / eviction counter deltas per step (finds start-up transients).

    python tools/diag_transient.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 5
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

KEYS = ("bytes_xfer_htd", "bytes_xfer_dth", "bytes_xfer_ctd", "bytes_xfer_dtc", "evictions", "evicted_bytes",
        "thrashing_detected", "revocations", "alloc_retries", "gpu_page_faults")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--simulate-tp", type=int, default=1)
    ap.add_argument("--tiers", default="host")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import importlib

    import torch
    importlib.import_module("open-gpu-kernel-modules_amd")
    from ogkm import rt
    from ogkm._native import lib
    from ogkm.models import llama

    rt.init("hip", host_budget_mb=0)
    # the emulated CXL pool, as bench.py: the NUMA node that is not the GPU's
    gpu_node = lib.device_numa_node(0)
    nodes = sorted({int(p.name[4:]) for p in Path("/sys/devices/system/node").glob("node[0-9]*")})
    other = [n for n in nodes if n != gpu_node]
    if not lib.cxl_info()["numa_nodes"] and other:
        lib.cxl_rediscover(other[0], "/sys")
    cfg = llama.CONFIGS[a.model]
    m = llama.TieredLlama(cfg, batch=64, context=1024, max_new_tokens=a.steps + 3, oversub=2.0, device=0,
                          tp_rank=0, tp_world=a.simulate_tp, seed=1234, lookahead=1, weight_format="ans",
                          tiers=a.tiers, kv_format="ans")
    tok = torch.randint(0, cfg.vocab, (64,)).cuda()
    for i in range(a.steps):
        s0 = lib.stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tok = m.step(tok)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s1 = lib.stats()
        d = {k: s1[k] - s0[k] for k in KEYS if k in s1}
        gb = {k: round(v / 1e9, 2) if "bytes" in k else v for k, v in d.items()}
        print(f"step {i}: {dt * 1e3:.1f} ms {gb}", flush=True)


if __name__ == "__main__":
    main()
