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

import torch

from .._native import lib


def _stream(t: torch.Tensor, dev: int) -> int:
    return int(torch.cuda.current_stream(dev).cuda_stream) if t.is_cuda else 0


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None,
             device_index: int = 0) -> torch.Tensor:
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.stride(1) != 1 or w.numel() != x.shape[1]:
        raise ValueError("rms_norm: x must be row-major bf16 [M, D] and w [D]")
    out = torch.empty_like(x) if out is None else out
    lib.rmsnorm(device_index, _stream(x, device_index), x.data_ptr(), w.data_ptr(), out.data_ptr(), x.shape[0],
                x.shape[1], x.stride(0), out.stride(0), float(eps))
    return out


def rope_kv(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, cache: torch.Tensor, pos: int, hq: int,
            hkv: int, tail: torch.Tensor | None = None, tail_pos: int = 0, device_index: int = 0) -> torch.Tensor:
    """qkv [B, (hq + 2 hkv) hd] -> rotated q [B, hq, hd]; rotated k and v are
    written into cache [2, B, hkv, T, hd] at ``pos`` (and into ``tail`` [2, B,
    hkv, tT, hd] at ``tail_pos`` when given)."""
    B = qkv.shape[0]
    hd = cache.shape[-1]
    T = cache.shape[-2]
    if qkv.stride(1) != 1 or cache.dtype != torch.bfloat16 or not cache.is_contiguous():
        raise ValueError("rope_kv: bad layout")
    if tail is not None and not tail.is_contiguous():
        raise ValueError("rope_kv: tail must be contiguous")
    q = torch.empty(B, hq, hd, dtype=torch.bfloat16, device=qkv.device)
    lib.rope_kv(device_index, _stream(qkv, device_index), qkv.data_ptr(), qkv.stride(0), cos.data_ptr(),
                sin.data_ptr(), q.data_ptr(), cache.data_ptr(), tail.data_ptr() if tail is not None else 0, B, hq,
                hkv, hd, T, pos, tail.shape[-2] if tail is not None else 0, tail_pos)
    return q


class _Work:
    buf: dict = {}


def attention(q: torch.Tensor, cache: torch.Tensor, length: int, device_index: int = 0) -> torch.Tensor:
    """q [B, hq, hd] (rotated), cache [2, B, hkv, T, hd] -> [B, hq * hd] bf16 over positions [0, length)."""
    B, hq, hd = q.shape
    hkv, T = cache.shape[2], cache.shape[3]
    nsplit = (length + 255) // 256
    need = B * hq * nsplit * (hd + 2) * 4
    key = str(q.device)
    ws = _Work.buf.get(key)
    if ws is None or ws.numel() * 4 < need:
        ws = torch.empty(max(need, 1 << 20) // 4 + 1024, dtype=torch.float32, device=q.device)
        _Work.buf[key] = ws
    out = torch.empty(B, hq * hd, dtype=torch.bfloat16, device=q.device)
    lib.attn_decode(device_index, _stream(q, device_index), q.data_ptr(), cache.data_ptr(), out.data_ptr(),
                    ws.data_ptr(), ws.numel() * 4, B, hq, hkv, hd, T, length, 1.0 / math.sqrt(hd))
    return out
