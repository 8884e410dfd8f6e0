#!/usr/bin/env python3
"""Decode-GEMM microbenchmark at Llama-3-70B decode shapes (M = batch): raw
bf16 fragment-order weights vs BF11-packed weights decoded in registers, for
each K unroll, and the staged alternative (k_bf12_unpack to bf16 + raw GEMM).
Prints one JSON line per variant."""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from ogkm import rt  # noqa: E402
from ogkm.ops import bf12, dgemm  # noqa: E402

SHAPES = ((10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672))
COLD = int(os.environ.get("COLD", "1"))
XFRAG = int(os.environ.get("XFRAG", "1"))  # activations in the GEMM's fragment order (as the model feeds them)
COLD_GB = float(os.environ.get("COLD_GB", "1.5"))
if os.environ.get("SHAPES"):  # e.g. "6144x4096,4096x4096,28672x4096,4096x14336" (Llama-3-8B)
    SHAPES = tuple(tuple(int(v) for v in s.split("x")) for s in os.environ["SHAPES"].split(","))


def timeit(fn, it=48):
    """GPU time per call from events around a captured HIP graph of `it` calls
    (no host launch overhead in the number; falls back to eager launches)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    try:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(it):
                    fn()
        run = g.replay
    except Exception:  # noqa: BLE001 - eager fallback
        def run():
            for _ in range(it):
                fn()
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / it


def main():
    m = int(os.environ.get("M", "64"))
    rt.init("hip", host_budget_mb=4096)
    ws = {}
    for n, k in SHAPES:
        w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
        flat = dgemm.frag_permute(w).contiguous()
        del w
        stream, info = bf12.pack(flat, fmt="bf11s")
        ws[(n, k)] = (flat, stream.cuda(), info, dgemm.packed_mode(stream))
    xs = {k: (torch.randn(m, k, device="cuda") * 0.5).to(torch.bfloat16) for _, k in SHAPES}
    stage = torch.empty(max(n * k for n, k in SHAPES), dtype=torch.bfloat16, device="cuda")
    variants = [("pipe", 0), ("pipe", 4)] + [("raw", u) for u in (2, 4)] + [("bf11", u) for u in (1, 2, 4)] + [("staged", 2)]
    if os.environ.get("VARIANTS"):  # e.g. "bf11:2,raw:2"
        variants = [(v.split(":")[0], int(v.split(":")[1])) for v in os.environ["VARIANTS"].split(",")]
    for kind, u in variants:
        # "pipe": the default raw split-K kernel (k_dgemm_pipe, UNROLL 0);
        # "raw": k_dgemm<RAW, u>
        dgemm.UNROLL = 0 if kind == "pipe" else u
        dgemm.PIPE = 1 if kind == "pipe" else 0
        # "pipe:D": the pipelined raw path at DEPTH D (0 = auto, 4 = k_dgemm_pipe,
        # 10 x slots = the LDS-ring k_dgemm_lring)
        dgemm.DEPTH = u if kind == "pipe" else 4
        tot_t, tot_b, per = 0.0, 0, {}
        for (n, k), (flat, pk, info, mode) in ws.items():
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            x = xs[k]
            if kind in ("raw", "pipe"):
                # COLD (default): rotate over enough weight copies (>= COLD_GB) that
                # no call finds its weights in the 256 MB MALL - as in a decode step,
                # where each layer's weights were last read one full step earlier
                ncopy = max(1, -(-int(COLD_GB * 2**30) // (n * k * 2))) if COLD else 1
                copies = [flat] + [flat.clone() for _ in range(ncopy - 1)]
                refs = [dgemm.WeightRef(c.data_ptr(), 0, n, k, dgemm.MODE_RAW) for c in copies]
                ctr = [0]

                xin, xr = (dgemm.to_frag(x), m) if XFRAG else (x, None)

                def fn(refs=refs, ctr=ctr, x=xin, out=out, xr=xr):
                    dgemm.linear(x, refs[ctr[0] % len(refs)], out=out, x_rows=xr)
                    ctr[0] += 1
                nb = n * k * 2
            elif kind == "bf11":
                ref = dgemm.WeightRef(pk.data_ptr(), 0, n, k, mode, 20)
                fn = lambda: dgemm.linear(x, ref, out=out)  # noqa: E731
                nb = info.nbytes
            else:
                ref = dgemm.WeightRef(stage.data_ptr(), 0, n, k, dgemm.MODE_RAW)

                def fn(pk=pk, info=info, ref=ref, out=out, x=x):
                    bf12.unpack_into(stage, pk.data_ptr(), info, 0)
                    dgemm.linear(x, ref, out=out)
                nb = info.nbytes
            dt = timeit(fn)
            copies = None
            per[f"{n}x{k}"] = round(dt * 1e3, 4)
            tot_t += dt
            tot_b += nb
        print(json.dumps({"variant": kind, "unroll": u, "M": m, "layer_ms": round(tot_t * 1e3, 3),
                          "weight_gbps": round(tot_b / tot_t / 1e9, 1), "per_shape_ms": per}), flush=True)


if __name__ == "__main__":
    main()
