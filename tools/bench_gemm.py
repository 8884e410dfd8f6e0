#!/usr/bin/env python3
"""Decode GEMM microbench: Y[M, N] = X[M, K] @ W[N, K]^T for the Llama-3-70B
decode shapes (M = batch), through each available path. Prints one JSON line
per (shape, path) with the effective weight-read bandwidth (the bound for
skinny GEMMs is HBM bytes of W)."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = {"wqkv": (10240, 8192), "wo": (8192, 8192), "wgu": (57344, 8192), "wd": (8192, 28672),
          "head": (128256, 8192)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--paths", default="matmul,linear,rocblas,ogkm")
    a = ap.parse_args()
    paths = a.paths.split(",")
    ogkm_gemm = None
    if "ogkm" in paths:
        try:
            import ogkm  # noqa: F401
            from ogkm.ops import gemm as ogkm_gemm
        except Exception as e:  # not built yet
            print(json.dumps({"path": "ogkm", "error": str(e)}))
            paths.remove("ogkm")
    for name, (n, k) in SHAPES.items():
        w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
        x = torch.randn(a.m, k, device="cuda").to(torch.bfloat16)
        ref = (x.float() @ w.float().t())
        for p in paths:
            if p == "matmul":
                torch.backends.cuda.preferred_blas_library("hipblaslt")
                fn = lambda: x @ w.t()  # noqa: E731
            elif p == "linear":
                torch.backends.cuda.preferred_blas_library("hipblaslt")
                fn = lambda: F.linear(x, w)  # noqa: E731
            elif p == "rocblas":
                torch.backends.cuda.preferred_blas_library("rocblas")
                fn = lambda: x @ w.t()  # noqa: E731
            elif p == "ogkm":
                fn = lambda: ogkm_gemm.linear(x, w)  # noqa: E731
            else:
                continue
            y = fn()
            err = float((y.float() - ref).abs().max() / ref.abs().max())
            dt = timeit(fn)
            print(json.dumps({"shape": name, "m": a.m, "n": n, "k": k, "path": p, "us": round(dt * 1e6, 1),
                              "weight_gbps": round(n * k * 2 / dt / 1e9, 1), "rel_err": round(err, 5)}), flush=True)
        torch.backends.cuda.preferred_blas_library("hipblaslt")
        del w, x, ref


if __name__ == "__main__":
    main()
