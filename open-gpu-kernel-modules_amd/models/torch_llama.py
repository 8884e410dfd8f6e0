"""A stock PyTorch Llama-3 decoder (torch.nn + aten ops only, no framework
calls) - the workload of the transparent managed mode.

``bench.py --torch-managed`` builds it under ``ogkm.managed()`` with the HBM
arena capped below the model + KV footprint, so the parameters and KV cache
oversubscribe HBM and the runtime moves them tensor by tensor as the
dispatcher declares them (SURVEY.md §7.1 design (1)); ``TieredLlama``
(models/llama.py) is the hand-planned engine for the same architecture.

Decode only: one token per sequence per step against a KV cache of
``context`` positions (prefilled with synthetic values), greedy sampling.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .llama import LlamaConfig


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float, dtype=torch.bfloat16):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim, dtype=dtype))
        self.eps = eps

    def forward(self, x):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).to(x.dtype) * self.weight


def rope(x, cos, sin):
    """x [B, H, hd] (rotate-half form), cos/sin [hd/2]."""
    x1, x2 = x[..., : x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
    return torch.cat([x1 * cos - x2 * sin, x1 * sin + x2 * cos], dim=-1)


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig, batch: int, context: int, dtype):
        super().__init__()
        hd = cfg.head_dim
        self.hq, self.hkv, self.hd = cfg.n_heads, cfg.n_kv_heads, hd
        self.attn_norm = RMSNorm(cfg.dim, cfg.norm_eps, dtype)
        self.wq = nn.Linear(cfg.dim, cfg.n_heads * hd, bias=False, dtype=dtype)
        self.wk = nn.Linear(cfg.dim, cfg.n_kv_heads * hd, bias=False, dtype=dtype)
        self.wv = nn.Linear(cfg.dim, cfg.n_kv_heads * hd, bias=False, dtype=dtype)
        self.wo = nn.Linear(cfg.n_heads * hd, cfg.dim, bias=False, dtype=dtype)
        self.ffn_norm = RMSNorm(cfg.dim, cfg.norm_eps, dtype)
        self.w1 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False, dtype=dtype)
        self.w3 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False, dtype=dtype)
        self.w2 = nn.Linear(cfg.ffn_dim, cfg.dim, bias=False, dtype=dtype)
        self.register_buffer("k_cache", torch.zeros(batch, cfg.n_kv_heads, context, hd, dtype=dtype), persistent=False)
        self.register_buffer("v_cache", torch.zeros(batch, cfg.n_kv_heads, context, hd, dtype=dtype), persistent=False)

    def forward(self, x, pos: int, cos, sin):
        B = x.shape[0]
        h = self.attn_norm(x)
        q = self.wq(h).view(B, self.hq, self.hd)
        k = self.wk(h).view(B, self.hkv, self.hd)
        v = self.wv(h).view(B, self.hkv, self.hd)
        q, k = rope(q, cos, sin), rope(k, cos, sin)
        self.k_cache[:, :, pos] = k
        self.v_cache[:, :, pos] = v
        kc, vc = self.k_cache[:, :, : pos + 1], self.v_cache[:, :, : pos + 1]
        a = F.scaled_dot_product_attention(q.unsqueeze(2), kc, vc, enable_gqa=True)  # [B, hq, 1, hd]
        x = x + self.wo(a.reshape(B, self.hq * self.hd))
        h = self.ffn_norm(x)
        return x + self.w2(F.silu(self.w1(h)) * self.w3(h))


class TorchLlama(nn.Module):
    def __init__(self, cfg: LlamaConfig, batch: int, context: int, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        self.embed = nn.Embedding(cfg.vocab, cfg.dim, dtype=dtype)
        self.layers = nn.ModuleList([Block(cfg, batch, context, dtype) for _ in range(cfg.n_layers)])
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps, dtype)
        self.head = nn.Linear(cfg.dim, cfg.vocab, bias=False, dtype=dtype)
        hd = cfg.head_dim
        inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
        ang = torch.outer(torch.arange(context, dtype=torch.float32), inv)
        self.register_buffer("cos", ang.cos().to(dtype), persistent=False)
        self.register_buffer("sin", ang.sin().to(dtype), persistent=False)

    @torch.no_grad()
    def step(self, tokens, pos: int):
        """One decode step: next greedy token of every sequence."""
        x = self.embed(tokens)
        cos, sin = self.cos[pos], self.sin[pos]
        for blk in self.layers:
            x = blk(x, pos, cos, sin)
        return self.head(self.norm(x)).argmax(-1)


def build_on_device(cfg: LlamaConfig, batch: int, context: int, device, std: float = 0.02, seed: int = 0,
                    prefill: int = 0) -> TorchLlama:
    """Random-init the model directly on ``device`` (no host copy of the weights:
    under the managed mode each parameter is created in HBM and may be evicted
    to host DRAM at once). The first ``prefill`` KV positions get synthetic
    values (the context a decode batch would have)."""
    with torch.device("meta"):
        m = TorchLlama(cfg, batch, context)
    m = m.to_empty(device=device)
    gen = torch.Generator(device=device).manual_seed(seed)
    hd = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float32, device=device) / hd))
    ang = torch.outer(torch.arange(context, dtype=torch.float32, device=device), inv)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith("norm.weight") or ".attn_norm." in name or ".ffn_norm." in name:
                p.fill_(1.0)
            else:
                p.normal_(0.0, std, generator=gen)
        m.cos.copy_(ang.cos())
        m.sin.copy_(ang.sin())
        for blk in m.layers:
            blk.k_cache.zero_()
            blk.v_cache.zero_()
            if prefill:
                blk.k_cache[:, :, :prefill].normal_(0.0, 1.0, generator=gen)
                blk.v_cache[:, :, :prefill].normal_(0.0, 1.0, generator=gen)
    return m


def footprint_bytes(cfg: LlamaConfig, batch: int, context: int) -> int:
    """bf16 bytes of parameters + KV cache."""
    kv = 2 * cfg.n_layers * batch * cfg.n_kv_heads * context * cfg.head_dim * 2
    return cfg.params() * 2 + kv


__all__ = ["TorchLlama", "build_on_device", "footprint_bytes", "rope"]
