"""Plain-PyTorch reference math of one Llama-3 decode step (bf16 / fp32).

These are the fp32 references the numerics tests compare the HIP kernels
against (llama.reference_step, tests/test_fused.py, tests/test_dgemm.py) and
the CPU path of the fake backend. The GPU decode itself runs the hand-written
gfx950 kernels: the MFMA decode GEMM (ops/dgemm.py, csrc/kernels/decode_gemm.hip)
and the fused RMSNorm / RoPE + KV append / GQA attention (ops/fused.py,
csrc/kernels/decode_ops.hip). The attention reference uses the grouped-query
layout directly (no KV repeat): q is viewed as [B, Hkv, group, hd] so each KV
head is read once.
"""
from __future__ import annotations

import math

import torch


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * w


def rope_tables(head_dim: int, max_pos: int, theta: float, device) -> tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64, device="cpu") / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [B, H, hd] at one position; cos/sin: [hd/2] (rotate-half convention)."""
    xf = x.float()
    h = xf.shape[-1] // 2
    x1, x2 = xf[..., :h], xf[..., h:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def gqa_decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, length: int) -> torch.Tensor:
    """q: [B, Hq, hd]; k/v_cache: [B, Hkv, T, hd]; attends to positions [0, length)."""
    B, Hq, hd = q.shape
    Hkv = k_cache.shape[1]
    g = Hq // Hkv
    k = k_cache[:, :, :length]
    v = v_cache[:, :, :length]
    qg = q.view(B, Hkv, g, hd)
    s = torch.matmul(qg, k.transpose(-1, -2)).float() * (1.0 / math.sqrt(hd))
    p = torch.softmax(s, dim=-1).to(q.dtype)
    o = torch.matmul(p, v)
    return o.reshape(B, Hq * hd)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.chunk(2, dim=-1)
    return torch.nn.functional.silu(g) * u
