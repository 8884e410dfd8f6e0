"""Fused decode-step ops (csrc/kernels/decode_ops.hip): one launch each where
the framework would issue 5-20 elementwise kernels. The fake backend runs the
C++ references of the same ops (csrc/core/dgemm_ref.cpp), so CPU tests exercise
the same plumbing (layouts, strides, positions).

  rms_norm(x, w, eps)                       RMSNorm, bf16 in/out, f32 math
  rope_kv(qkv, cos, sin, cache, pos, ...)   RoPE on q/k + append k/v into the KV cache (+ a tail copy)
  attention(q, cache, length)               GQA decode attention, split over the context
"""
from __future__ import annotations

import math
import os

import torch

from .._native import lib


def _stream(t: torch.Tensor, dev: int) -> int:
    return int(torch.cuda.current_stream(dev).cuda_stream) if t.is_cuda else 0


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None,
             device_index: int = 0, pending=None, out_frag: bool = False) -> torch.Tensor:
    """RMSNorm of x [M, D]. ``pending`` (a dgemm.Deferred [M, D] GEMM): first
    x += bf16(its split-K sum), in place - its residual epilogue - in the same
    launch (bit-identical to linear(..., "resid") followed by rms_norm).
    ``out_frag``: the output is the decode GEMM's fragment-ordered activation
    buffer [frag_rows(M), D] (dgemm.to_frag layout)."""
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.stride(1) != 1 or w.numel() != x.shape[1]:
        raise ValueError("rms_norm: x must be row-major bf16 [M, D] and w [D]")
    if out is None:
        out = (torch.empty((x.shape[0] + 15) // 16 * 16, x.shape[1], dtype=x.dtype, device=x.device) if out_frag
               else torch.empty_like(x))
    part, ks = 0, 0
    if pending is not None:
        pending.check(x.shape[0], x.shape[1])
        part, ks = pending.part, pending.ksplit
    ssq, ssq_bytes = 0, 0
    if WIDE_NORM and x.device.type == "cuda":
        need = x.shape[0] * ((x.shape[1] + 1023) // 1024) * 4
        key = str(x.device)
        t = _NormScratch.buf.get(key)
        if t is None or t.numel() * 4 < need:
            t = _NormScratch.buf[key] = torch.empty(max(need, 1 << 16) // 4, dtype=torch.float32, device=x.device)
        ssq, ssq_bytes = t.data_ptr(), t.numel() * 4
    lib.rmsnorm(device_index, _stream(x, device_index), x.data_ptr(), w.data_ptr(), out.data_ptr(), x.shape[0],
                x.shape[1], x.stride(0), out.stride(0), float(eps), part, ks, out_frag, ssq, ssq_bytes)
    return out


# Few-row norms as two wide launches (k_norm_ssq + k_norm_scale) instead of one
# workgroup per row (OGKM_WIDE_NORM=1). Off by default: measured 5.1 + 5.1 us
# per norm on config 2 against the one-launch kernel's 8.5 (profiles/r4_config2.md).
WIDE_NORM = os.environ.get("OGKM_WIDE_NORM", "0") != "0"


class _NormScratch:
    buf: dict = {}


def rope_kv(qkv, cos: torch.Tensor, sin: torch.Tensor, cache: torch.Tensor, pos: int, hq: int,
            hkv: int, tail: torch.Tensor | None = None, tail_pos: int = 0, device_index: int = 0) -> torch.Tensor:
    """qkv [B, (hq + 2 hkv) hd] -> rotated q [B, hq, hd]; rotated k and v are
    written into cache [2, B, hkv, T, hd] at ``pos`` (and into ``tail`` [2, B,
    hkv, tT, hd] at ``tail_pos`` when given). ``qkv`` may be a dgemm.Deferred:
    the kernel then sums its K splits (the GEMM's store epilogue) itself."""
    hd = cache.shape[-1]
    T = cache.shape[-2]
    if cache.dtype != torch.bfloat16 or not cache.is_contiguous():
        raise ValueError("rope_kv: bad layout")
    if tail is not None and not tail.is_contiguous():
        raise ValueError("rope_kv: tail must be contiguous")
    part, ks = 0, 0
    if isinstance(qkv, torch.Tensor):
        if qkv.stride(1) != 1:
            raise ValueError("rope_kv: bad layout")
        B, ptr, ld = qkv.shape[0], qkv.data_ptr(), qkv.stride(0)
    else:
        B = qkv.m
        qkv.check(B, (hq + 2 * hkv) * hd)
        part, ks, ptr, ld = qkv.part, qkv.ksplit, 0, 0
    q = torch.empty(B, hq, hd, dtype=torch.bfloat16, device=cache.device)
    lib.rope_kv(device_index, _stream(cache, device_index), ptr, ld, cos.data_ptr(),
                sin.data_ptr(), q.data_ptr(), cache.data_ptr(), tail.data_ptr() if tail is not None else 0, B, hq,
                hkv, hd, T, pos, tail.shape[-2] if tail is not None else 0, tail_pos, part, ks)
    return q


class _Work:
    buf: dict = {}


def attention(q: torch.Tensor, cache: torch.Tensor, length: int, device_index: int = 0,
              out_frag: bool = False, split_tokens: int = 0) -> torch.Tensor:
    """q [B, hq, hd] (rotated), cache [2, B, hkv, T, hd] -> [B, hq * hd] bf16 over positions [0, length)
    (``out_frag``: the decode GEMM's fragment-ordered [frag_rows(B), hq * hd] buffer)."""
    B, hq, hd = q.shape
    hkv, T = cache.shape[2], cache.shape[3]
    nsplit = (length + 63) // 64  # upper bound (split_tokens 64)
    need = B * hq * nsplit * (hd + 2) * 4
    key = str(q.device)
    ws = _Work.buf.get(key)
    if ws is None or ws.numel() * 4 < need:
        ws = torch.empty(max(need, 1 << 20) // 4 + 1024, dtype=torch.float32, device=q.device)
        _Work.buf[key] = ws
    out = torch.empty((B + 15) // 16 * 16 if out_frag else B, hq * hd, dtype=torch.bfloat16, device=q.device)
    lib.attn_decode(device_index, _stream(q, device_index), q.data_ptr(), cache.data_ptr(), out.data_ptr(),
                    ws.data_ptr(), ws.numel() * 4, B, hq, hkv, hd, T, length, 1.0 / math.sqrt(hd), out_frag,
                    split_tokens)
    return out
