"""Tensor-parallel (Megatron-style) sharding of Llama weights.

Column-parallel: QKV (by heads) and gate/up (by FFN columns) - each rank owns a
slice of the output features, no communication. Row-parallel: O and down - each
rank owns a slice of the input features; the partial outputs are all-reduced
over RCCL (2 all-reduces per layer). The vocab projection is column-parallel and
the greedy token is chosen by an all-gather of per-rank (max, argmax) pairs.

For decode at 2x oversubscription, TP is also the *bandwidth* lever: every rank
streams only its 1/N of the non-resident weights over its own PCIe link, so the
aggregate host->HBM bandwidth grows with N while the per-step bytes per GPU
shrink.
"""
from __future__ import annotations

import torch

from . import comm


def shard_rows(w: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Column-parallel shard: split the output features (rows of [out, in])."""
    n = w.shape[0] // world
    return w[rank * n:(rank + 1) * n]


def shard_cols(w: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Row-parallel shard: split the input features (columns of [out, in])."""
    n = w.shape[1] // world
    return w[:, rank * n:(rank + 1) * n]


def shard_qkv(wq: torch.Tensor, wk: torch.Tensor, wv: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    return torch.cat([shard_rows(wq, rank, world), shard_rows(wk, rank, world), shard_rows(wv, rank, world)], 0)


def shard_gate_up(wg: torch.Tensor, wu: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    return torch.cat([shard_rows(wg, rank, world), shard_rows(wu, rank, world)], 0)


def row_parallel_reduce(y: torch.Tensor) -> torch.Tensor:
    return comm.all_reduce_(y)


def vocab_parallel_argmax(logits_local: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Greedy token over a vocab sharded across ranks: [B, V/world] -> [B]."""
    val, idx = logits_local.float().max(dim=-1)
    if world == 1:
        return idx
    idx = idx + rank * logits_local.shape[-1]
    pair = torch.stack([val, idx.to(torch.float32)], dim=-1)  # [B, 2]
    allp = comm.all_gather_cat(pair.unsqueeze(0), dim=0)      # [world, B, 2]
    best = allp[..., 0].argmax(dim=0)                          # [B]
    return allp[..., 1].gather(0, best.unsqueeze(0)).squeeze(0).to(torch.int64)
