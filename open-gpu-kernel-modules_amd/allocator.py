"""PyTorch pluggable allocator backed by the runtime's HBM arena.

``enable()`` routes every torch CUDA allocation through
``ogkm_torch_alloc`` / ``ogkm_torch_free`` (csrc/core/torch_allocator.cpp), so
model tensors and managed ranges share one HBM budget (north-star config 2:
"allocator baseline"). Must be called before the first CUDA allocation.

Frees are stream-ordered: the freeing stream's fence guards the memory, and
the next allocation of it makes its own stream wait for that fence GPU-side
(csrc/core/torch_allocator.cpp).

Managed mode (``enable(managed_min_mb=N)``): allocations of at least N MB are
runtime-managed ranges at a stable device VA (HIP VMM), so torch tensors
oversubscribe HBM. A tensor is active (resident, pinned) until :func:`park`;
parked tensors are evictable by the arena LRU (to host DRAM) and
:func:`unpark` brings them back at the same address, the current stream waiting
GPU-side for the copies - the cudaMallocManaged + cudaMemPrefetchAsync pattern
(reference: uvm_migrate.c) with explicit park points, since a kernel touching
an evicted tensor would hit an unmapped VA (no replayable faults without XNACK).
"""
from __future__ import annotations

import contextlib

from ._native import SO_PATH, lib

_enabled = False


def enable(managed_min_mb: int = 0) -> None:
    """Route torch CUDA allocations through the runtime. ``managed_min_mb`` > 0
    turns on managed mode for allocations of at least that many MB (call before
    the runtime creates its HBM arena: it selects the VMM arena provider)."""
    global _enabled
    if _enabled:
        return
    import torch

    if managed_min_mb > 0:
        lib.configure("hbm_provider", 1)
        lib.configure("torch_alloc_managed_min_mb", int(managed_min_mb))

    alloc = torch.cuda.memory.CUDAPluggableAllocator(str(SO_PATH), "ogkm_torch_alloc", "ogkm_torch_free")
    torch.cuda.memory.change_current_allocator(alloc)
    _enabled = True


def enabled() -> bool:
    return _enabled


def empty_cache(device: int = 0) -> None:
    """Hand the freed memory the allocator caches for reuse (extents, empty
    slabs) back to the runtime's HBM arena - torch.cuda.empty_cache()'s role."""
    lib.torch_alloc_trim(device)


def stats(device: int = 0) -> dict:
    a, p, n, w = lib.torch_alloc_stats(device)[:4]
    return {"allocated": a, "peak": p, "allocs": n, "stream_waits": w}


def _base(t) -> tuple[int, int]:
    """(allocation base pointer, device) of a CUDA tensor."""
    return t.untyped_storage().data_ptr(), t.device.index or 0


def _stream(dev: int) -> int:
    import torch

    return torch.cuda.current_stream(dev).cuda_stream


def park(*tensors) -> None:
    """Mark managed tensors evictable; their queued uses on the current stream
    fence any eviction. Do not touch a parked tensor before :func:`unpark`."""
    for t in tensors:
        p, d = _base(t)
        lib.torch_park(p, d, _stream(d))


def unpark(*tensors) -> None:
    """Make parked tensors resident again (same addresses); the current stream
    waits GPU-side for the copies, the host does not."""
    for t in tensors:
        p, d = _base(t)
        lib.torch_unpark(p, d, _stream(d))


@contextlib.contextmanager
def parked(*tensors):
    """``with parked(a, b): ...`` - a and b may be evicted inside the block."""
    park(*tensors)
    try:
        yield
    finally:
        unpark(*tensors)


def set_read_mostly(*tensors, on: bool = True) -> None:
    """Managed tensors that are only read keep their host copy while resident
    in HBM (READ_MOSTLY / read duplication): evicting them costs no copy-out."""
    for t in tensors:
        p, d = _base(t)
        lib.torch_set_read_mostly(p, d, on)


def advise(t, advice: int, loc=None, proc: int | None = None) -> None:
    """cudaMemAdvise on a managed tensor (``advice`` = rt.ADVISE_*; ``loc`` as
    in rt.mem_advise, e.g. "gpu:0" / "host:1" / "cxl:2"; ``proc`` the accessing
    processor for SET_ACCESSED_BY). Under ``ogkm.managed()`` a decision to
    access the tensor remotely (accessed_by, a thrashing pin) is served by a
    local copy: the tensor's device address maps HBM only."""
    from .rt import CPU, Loc

    p, d = _base(t)
    kind, i = Loc.parse(loc).code if loc is not None else (0, d)
    lib.torch_advise(p, d, int(advice), int(kind), int(i), d if proc is None else (CPU if proc == "cpu" else int(proc)))


def last_error(device: int = 0) -> str:
    """Why the last allocation on ``device`` failed (empty: it did not)."""
    return lib.torch_last_error(device)


def is_managed(t) -> bool:
    p, d = _base(t)
    return lib.torch_is_managed(p, d)


def park_all(device: int = 0) -> None:
    """Drop the allocation hold of every managed tensor of ``device``."""
    lib.torch_park_all(device, _stream(device))


def managed_stats(device: int = 0) -> dict:
    return lib.torch_managed_stats(device)
