"""Peer-memory client: expose runtime memory to third-party importers (NICs,
other processes, other GPUs) - the nvidia-peermem / nvidia_p2p_* analog.

Reference behaviour:
  * ``nvidia_p2p_get_pages`` pins a 64 KB-aligned GPU VA range and returns a page
    table of 64 KB pages (kernel-open/nvidia/nv-p2p.c:362-942, alignment check
    :421-431, page sizes nv-p2p.h:115-119); ``put_pages`` unpins it.
  * nvidia-peermem's ``acquire`` probes a range with get/put (pm/nvidia-peermem.c:
    198-243), ``get_pages`` pins (:397-425), ``dma_map`` builds a scatter list of
    the pinned pages (:245-300), and a free callback invalidates the importer's
    mapping when the owner frees the memory (:129-180). A "persistent" client
    (:446-488) pins without a callback.
  * dma-buf export of GPU memory (kernel-open/nvidia/nv-dmabuf.c:1084-1100,1360).

MI355X design: there is no kernel pinning to do. A region of a managed buffer is
pinned by a runtime *lease* on the exporting GPU (the chunk cannot be evicted or
relocated while the lease lives - the arena pin count, arena.cpp), and the
device pointer is handed out as

  * a 64 KB page table / coalesced segment list (``pages()`` / ``dma_map()``),
  * a dma-buf fd (``export_dmabuf`` -> ``hsa_amd_portable_export_dmabuf``; what
    RDMA NICs import on ROCm), or
  * a HIP IPC handle (``ipc_handle`` / ``open_ipc``) for another process on the
    node, which then reads the peer's HBM directly over xGMI.

On the fake backend the "HBM" is a shared memfd, so export and IPC are real
file-descriptor sharing between processes (tests/test_p2p.py).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Callable, Optional

from . import rt
from ._native import lib

P2P_PAGE_SIZE = 64 << 10  # the reference's GPU page size for third-party mappings

__all__ = ["P2P_PAGE_SIZE", "PeerRegion", "PeerMemClient", "IpcMapping", "open_ipc", "default_client"]


@dataclass
class PeerRegion:
    """A pinned, exported region (nvidia_p2p_page_table analog)."""

    client: "PeerMemClient"
    buf: rt.ManagedBuffer
    offset: int
    nbytes: int
    device: int
    dptr: int
    page_size: int
    free_callback: Optional[Callable[["PeerRegion"], None]]
    _lease: Optional[rt.Lease] = None
    valid: bool = True
    _fds: list = field(default_factory=list)

    @property
    def npages(self) -> int:
        return (self.nbytes + self.page_size - 1) // self.page_size

    def pages(self) -> list[int]:
        """Device address of every page of the region (get_pages' page table)."""
        self._check()
        return [self.dptr + i * self.page_size for i in range(self.npages)]

    def dma_map(self) -> list[tuple[int, int]]:
        """Scatter list: physically/virtually contiguous page runs coalesced into
        (address, length) segments. A runtime lease is one contiguous extent, so
        this is a single segment (the reference builds one sg entry per page)."""
        self._check()
        segs: list[tuple[int, int]] = []
        for p in self.pages():
            ln = min(self.page_size, self.dptr + self.nbytes - p)
            if segs and segs[-1][0] + segs[-1][1] == p:
                segs[-1] = (segs[-1][0], segs[-1][1] + ln)
            else:
                segs.append((p, ln))
        return segs

    def export_dmabuf(self) -> tuple[int, int]:
        """(fd, offset of dptr inside the exported buffer). The caller owns the fd."""
        self._check()
        fd, off = lib.export_dmabuf(self.dptr, self.nbytes)
        return fd, off

    def ipc_handle(self) -> bytes:
        """Handle another process on the node opens with ``open_ipc``."""
        self._check()
        return lib.ipc_handle(self.dptr)

    def tensor(self, shape, dtype):
        self._check()
        return self._lease.tensor(shape, dtype)

    def put(self) -> None:
        """put_pages: drop the pin (idempotent)."""
        self.client.put_pages(self)

    def _check(self) -> None:
        if not self.valid:
            raise RuntimeError("peer region was invalidated (its memory was freed or put)")


class PeerMemClient:
    """One importer registration (an ib_core peer-memory client analog).

    ``persistent=True`` mirrors the reference's NC client: regions carry no free
    callback and freeing pinned memory fails with BUSY until they are put.
    Otherwise freeing the owner invalidates the region and runs its callback
    (the owner-driven revocation of nv-p2p's free callback)."""

    def __init__(self, name: str = "ogkm-peermem", persistent: bool = False, page_size: int = P2P_PAGE_SIZE):
        if page_size not in (4 << 10, 64 << 10, 128 << 10, 2 << 20):
            raise ValueError("page_size must be 4K, 64K, 128K or 2M")
        self.name = name
        self.persistent = persistent
        self.page_size = page_size
        self._regions: dict[int, list[PeerRegion]] = {}
        self._m = threading.Lock()
        self.stats = {"acquire": 0, "get_pages": 0, "put_pages": 0, "invalidations": 0}
        rt._free_hooks.append(self._on_free)

    def close(self) -> None:
        for regs in list(self._regions.values()):
            for r in list(regs):
                self.put_pages(r)
        if self._on_free in rt._free_hooks:
            rt._free_hooks.remove(self._on_free)

    # -- probing
    def acquire(self, buf: rt.ManagedBuffer, offset: int = 0, nbytes: Optional[int] = None, device: int = 0) -> bool:
        """Is [offset, offset+nbytes) exportable from ``device``? Probes with a
        get/put pair like nvidia-peermem's acquire."""
        self.stats["acquire"] += 1
        nbytes = buf.size - offset if nbytes is None else nbytes
        if offset % self.page_size or nbytes <= 0 or offset + nbytes > buf.size:
            return False
        try:
            self.put_pages(self.get_pages(buf, offset, nbytes, device))
        except (RuntimeError, ValueError):
            return False
        return True

    # -- pin / unpin
    def get_pages(self, buf: rt.ManagedBuffer, offset: int = 0, nbytes: Optional[int] = None, device: int = 0,
                  free_callback: Optional[Callable[[PeerRegion], None]] = None) -> PeerRegion:
        nbytes = buf.size - offset if nbytes is None else nbytes
        if offset % self.page_size:
            raise ValueError(f"offset must be {self.page_size}-byte aligned (nv-p2p.c:421-431)")
        if nbytes <= 0 or offset + nbytes > buf.size:
            raise ValueError("region outside the buffer")
        if self.persistent and free_callback is not None:
            raise ValueError("persistent clients take no free callback")
        foreign = lib.range_info(buf.id)["type"] in ("external", "device_p2p")
        # The lease is the pin: the extent cannot be evicted or relocated while it lives.
        lease = buf.acquire(device, rt.WRITE, offset, nbytes)
        lease.wait(0)
        if lease.remote and not foreign:
            lease.release(0)
            raise RuntimeError("region is only remotely mapped on this device; cannot export")
        dptr = lease.dptr
        reg = PeerRegion(self, buf, offset, nbytes, device, dptr, self.page_size, free_callback, lease)
        with self._m:
            self._regions.setdefault(buf.id, []).append(reg)
        self.stats["get_pages"] += 1
        return reg

    def put_pages(self, reg: PeerRegion) -> None:
        with self._m:
            regs = self._regions.get(reg.buf.id, [])
            if reg in regs:
                regs.remove(reg)
            if not regs:
                self._regions.pop(reg.buf.id, None)
        if reg.valid:
            reg.valid = False
            if reg._lease is not None:
                reg._lease.release(0)
                reg._lease = None
            self.stats["put_pages"] += 1

    def regions(self, buf: Optional[rt.ManagedBuffer] = None) -> list[PeerRegion]:
        with self._m:
            if buf is not None:
                return list(self._regions.get(buf.id, []))
            return [r for v in self._regions.values() for r in v]

    # -- owner-side free -> importer invalidation
    def _on_free(self, buf: rt.ManagedBuffer) -> None:
        regs = self.regions(buf)
        if not regs:
            return
        if self.persistent:
            raise RuntimeError(f"buffer {buf.id} is pinned by persistent peer client {self.name!r}; put it first")
        for r in regs:
            cb = r.free_callback
            self.put_pages(r)
            self.stats["invalidations"] += 1
            if cb is not None:
                cb(r)


class IpcMapping:
    """Another process's exported region mapped into this one (peer HBM over
    xGMI on a GPU box). ``close()`` unmaps it."""

    def __init__(self, handle: bytes, nbytes: int, device: int = 0):
        self.ptr = lib.ipc_open(handle)
        self.nbytes = nbytes
        self.device = device
        self._open = True

    def tensor(self, shape, dtype):
        dev = "cpu" if lib.backend_name() == "fake" else "cuda"
        return rt._tensor_from_ptr(self.ptr, shape, dtype, dev, self.device, 0)

    def close(self) -> None:
        if self._open:
            lib.ipc_close(self.ptr)
            self._open = False

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def open_ipc(handle: bytes, nbytes: int, device: int = 0) -> IpcMapping:
    return IpcMapping(handle, nbytes, device)


_default: Optional[PeerMemClient] = None


def default_client() -> PeerMemClient:
    global _default
    if _default is None:
        _default = PeerMemClient()
    return _default


class DmabufImport:
    """Importer side of a dma-buf fd (from ``export_dmabuf`` here or in another
    process, or a third-party exporter): the buffer mapped into a GPU's address
    space (``hsa_amd_interop_map_buffer``). ``tensor()`` views it for kernels;
    the mapping is device-visible only (the HIP runtime does not track it, so
    hipMemcpy / ``.cpu()`` cannot read it - use kernels or the runtime's ring
    copies). ``close()`` unmaps. The consumer half of the peer-memory contract (nvidia-peermem's
    importer role, kernel-open/nvidia-peermem/nvidia-peermem.c)."""

    def __init__(self, fd: int, device: int = 0):
        self.fd = fd
        self.device = device
        self.ptr, self.nbytes = lib.import_dmabuf(device, fd)

    def tensor(self, shape, dtype, offset: int = 0):
        from .rt import _tensor_from_ptr
        dev = "cpu" if lib.backend_name() == "fake" else "cuda"
        return _tensor_from_ptr(self.ptr + offset, shape, dtype, dev, self.device)

    def close(self) -> None:
        if self.ptr:
            lib.unimport_dmabuf(self.ptr)
            self.ptr = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
