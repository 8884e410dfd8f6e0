"""PyTorch pluggable allocator backed by the runtime's HBM arena.

``enable()`` routes every torch CUDA allocation through
``ogkm_torch_alloc`` / ``ogkm_torch_free`` (csrc/core/torch_allocator.cpp), so
model tensors and managed ranges share one HBM budget (north-star config 2:
"allocator baseline"). Must be called before the first CUDA allocation.

Frees are stream-ordered: the freeing stream's fence guards the memory, and
the next allocation of it makes its own stream wait for that fence GPU-side
(csrc/core/torch_allocator.cpp).
"""
from __future__ import annotations

from ._native import SO_PATH, lib

_enabled = False


def enable() -> None:
    global _enabled
    if _enabled:
        return
    import torch

    alloc = torch.cuda.memory.CUDAPluggableAllocator(str(SO_PATH), "ogkm_torch_alloc", "ogkm_torch_free")
    torch.cuda.memory.change_current_allocator(alloc)
    _enabled = True


def enabled() -> bool:
    return _enabled


def stats(device: int = 0) -> dict:
    a, p, n, w = lib.torch_alloc_stats(device)
    return {"allocated": a, "peak": p, "allocs": n, "stream_waits": w}
