"""Python entry points to the migration data-plane kernels
(csrc/kernels/copy_kernels.hip): batched copies on a ring, page-list pack/unpack,
and the residency-checking gather used for host-resident embedding tables.
"""
from __future__ import annotations

import torch

from .._native import lib
from .. import rt

RING_CPU_TO_GPU, RING_GPU_TO_CPU, RING_GPU_INTERNAL, RING_GPU_TO_GPU, RING_MEMOPS, RING_CXL = range(6)


def ring_copy(dst: int, src: int, nbytes: int, device: int = 0, ring: int = RING_GPU_INTERNAL, wait: bool = True):
    """Copy through a migration ring (one k_batch_copy launch + tracking release)."""
    return lib.ring_copy(device, ring, dst, src, nbytes, wait)


def gather_pages(src: torch.Tensor, dst: torch.Tensor, pages: list[int], page_bytes: int = 4096, device: int = 0):
    """Pack pages ``pages`` of ``src`` into contiguous ``dst`` (k_gather_pages)."""
    lib.ring_gather(device, src.data_ptr(), dst.data_ptr(), list(pages), page_bytes, False)


def scatter_pages(dst: torch.Tensor, src: torch.Tensor, pages: list[int], page_bytes: int = 4096, device: int = 0):
    """Unpack contiguous ``src`` into pages ``pages`` of ``dst`` (k_scatter_pages)."""
    lib.ring_gather(device, dst.data_ptr(), src.data_ptr(), list(pages), page_bytes, True)


def managed_embedding(table: "rt.ManagedBuffer", ids: torch.Tensor, dim: int, dtype=torch.bfloat16,
                      device: int = 0) -> torch.Tensor:
    """Rows ``ids`` of a managed [vocab, dim] table.

    HIP backend: k_managed_gather reads each row where it lives (HBM if resident,
    else host/CXL over PCIe - the UVM "accessed_by + remote mapping" case) and
    records misses / remote accesses in the device fault buffer for the access
    counters. Fake backend: a remote lease + index_select on the host view.
    """
    esz = torch.empty((), dtype=dtype).element_size()
    if lib.backend_name() == "fake":
        lease = table.acquire(device, rt.READ)
        lease.wait(0)
        t = lease.tensor((table.size // (dim * esz), dim), dtype)
        out = t.index_select(0, ids.to(torch.int64).cpu()).clone()
        lease.release(0)
        return out
    ids = ids.to(device=f"cuda:{device}", dtype=torch.int64).contiguous()
    out = torch.empty(ids.numel(), dim, dtype=dtype, device=f"cuda:{device}")
    lib.managed_gather(table.id, ids.data_ptr(), ids.numel(), dim * esz, out.data_ptr(), device,
                       torch.cuda.current_stream(device).cuda_stream)
    return out
