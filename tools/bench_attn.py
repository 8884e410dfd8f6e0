#!/usr/bin/env python3
"""Decode-attention microbenchmark (k_attn_decode_ws + combine): one layer's KV
at the bench shapes, time per call and effective KV-read bandwidth.
    python tools/bench_attn.py            (GRAPH=0: eager calls, SPLIT=64|256, COLD=0, SHAPE=70b-tp8)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm.ops import fused  # noqa: E402

SHAPES = {  # name: (B, hq, hkv, hd, len)
    "8b": (64, 32, 8, 128, 1025),
    "70b": (64, 64, 8, 128, 1025),
    "70b-tp8": (64, 8, 1, 128, 1025),
    "405b-tp8": (64, 16, 1, 128, 1025),
}


def main() -> None:
    rt.init("hip")
    iters = int(os.environ.get("ITERS", "50"))
    graph = int(os.environ.get("GRAPH", "1"))  # 0: back-to-back eager calls (includes host launch cost)
    only = os.environ.get("SHAPE")  # one shape (profiling runs)
    for name, (B, hq, hkv, hd, L) in SHAPES.items():
        if only and name != only:
            continue
        T = L
        q = torch.randn(B, hq, hd, device="cuda").to(torch.bfloat16)
        # MALL-cold: rotate over >= 1 GB of caches (a decode step reads every
        # layer's KV once; one layer's KV re-read would sit in the 256 MB MALL)
        kvb = 2 * B * hkv * T * hd * 2
        ncopy = max(1, -(-(1 << 30) // kvb)) if int(os.environ.get("COLD", "1")) else 1
        caches = [torch.randn(2, B, hkv, T, hd, device="cuda").to(torch.bfloat16) for _ in range(ncopy)]
        st = int(os.environ.get("SPLIT", "0"))  # 0 auto, 64, 256
        for i in range(3):
            fused.attention(q, caches[i % ncopy], L, split_tokens=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if graph:
            # GPU time only: the calls captured once into a graph and replayed
            # (a one-KV-head layer's KV is ~33 MB, ~10 us - less than the
            # host-side launch cost of one call)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(iters):
                    fused.attention(q, caches[i % ncopy], L, split_tokens=st)
            g.replay()
            torch.cuda.synchronize()
            e0.record()
            g.replay()
            e1.record()
        else:
            e0.record()
            for i in range(iters):
                fused.attention(q, caches[i % ncopy], L, split_tokens=st)
            e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        gb = 2 * B * hkv * L * hd * 2 / 1e9
        print(f"{name:9s} B={B} hq={hq} hkv={hkv} hd={hd} len={L} {us:8.1f} us  "
              f"KV {gb * 1e3:7.1f} MB  {gb / (us * 1e-6):7.0f} GB/s  split {st or 'auto'}  {'graph' if graph else 'eager'}",
              flush=True)
        del caches


if __name__ == "__main__":
    main()
