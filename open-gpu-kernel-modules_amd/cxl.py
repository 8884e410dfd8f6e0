"""CXL.mem tier API (capabilities of the CXLMemUring fork).

  get_info()          <- NV2080_CTRL_CMD_BUS_GET_CXL_INFO      (kern_bus_ctrl.c:745-781)
  register_buffer()   <- ..._REGISTER_CXL_BUFFER              (kern_bus_ctrl.c:785-836, p2p_cxl.c:226-353)
  unregister_buffer() <- ..._UNREGISTER_CXL_BUFFER            (kern_bus_ctrl.c:839-870; unreachable there, works here)
  dma()               <- ..._CXL_P2P_DMA_REQUEST              (kern_bus_ctrl.c:873-932, p2p_cxl.c:517-677)
  pages()/put_pages() <- RmP2PGetCxlPages / PutCxlPages       (p2p_cxl.c:424-507)
  p2p_caps()          <- P2P caps CXL bit                     (ctrl0000system.h:1085-1147)

Differences by design: handles are generation-checked opaque ids (never kernel
pointers), GPU memory is addressed by device pointer (never a raw FB offset),
DMA is asynchronous through the runtime's CXL ring with real transfer ids, and
``measure_bandwidth`` reports measured GB/s instead of a hard-coded 3900 MBps.
When the machine has no CXL device, a NUMA node can be *emulated* as the CXL
pool (config ``cxl_emulate_node``) - results are then labelled ``emulated``.
"""
from __future__ import annotations

import ctypes
import os
import ctypes.util
import mmap
import time
from typing import Iterable, Optional

from ._native import lib

DIR_GPU_TO_CXL = 0
DIR_CXL_TO_GPU = 1


def get_info() -> dict:
    return lib.cxl_info()


def rediscover(emulate_node: int = -1, sysfs_root: str = "/sys", emulate_nodes: Iterable[int] = ()) -> dict:
    """Re-scan CXL memory. Without CXL hardware, ``emulate_node`` / every node in
    ``emulate_nodes`` stands in for a CXL pool (one per socket lets every rank
    demote to the pool on its own socket: ``lib.cxl_nearest_node``)."""
    mask = 0
    for n in emulate_nodes:
        mask |= 1 << int(n)
    lib.cxl_rediscover(emulate_node, sysfs_root, mask)
    return lib.cxl_info()


class CxlBuffer:
    """A registered CXL (or CXL-emulating) host buffer."""

    def __init__(self, base: int, size: int, version: int = 2, owner=None):
        self.base = base
        self.size = size
        self.handle = lib.cxl_register(base, size, version)
        self._owner = owner  # keeps an mmap alive

    @staticmethod
    def allocate(size: int, version: int = 2, node: Optional[int] = None) -> "CxlBuffer":
        """Allocate page-aligned memory (bound to ``node`` when given) and register it."""
        m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        base = ctypes.addressof(ctypes.c_char.from_buffer(m))
        if node is not None:
            _mbind(base, size, node)
        # touch to populate on the bound node
        ctypes.memset(base, 0, size)
        return CxlBuffer(base, size, version, owner=m)

    def info(self) -> dict:
        return lib.cxl_buffer(self.handle)

    def pages(self, offset: int = 0, length: Optional[int] = None) -> list[tuple[int, int]]:
        return lib.cxl_pages(self.handle, offset, self.size - offset if length is None else length)

    def put_pages(self) -> None:
        lib.cxl_put_pages(self.handle)

    def dma(self, gpu_ptr: int, device: int, offset: int, nbytes: int, direction: int, async_: bool = True) -> int:
        return lib.cxl_dma(self.handle, gpu_ptr, device, offset, nbytes, direction, async_)

    def unregister(self) -> None:
        if self.handle:
            lib.cxl_unregister(self.handle)
            self.handle = 0

    def __del__(self):
        try:
            if self.handle and lib.is_initialized():
                self.unregister()
        except Exception:
            pass


def wait(transfer_id: int) -> None:
    lib.cxl_dma_wait(transfer_id)


def _mbind(addr: int, size: int, node: int) -> None:
    libc = ctypes.CDLL(None, use_errno=True)
    try:
        mbind = libc.mbind
    except AttributeError:
        mbind = ctypes.CDLL(ctypes.util.find_library("numa")).mbind
    mask = ctypes.c_ulong(1 << node)
    MPOL_BIND = 2
    mbind.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int, ctypes.POINTER(ctypes.c_ulong), ctypes.c_ulong,
                      ctypes.c_uint]
    mbind(addr, size, MPOL_BIND, ctypes.byref(mask), 64, 0)


def numa_distances(node: int, sysfs: str = "/sys") -> dict:
    """SLIT distances from NUMA ``node`` to every node ({node: distance}), from
    ``<sysfs>/devices/system/node/node<N>/distance`` ({} when unreadable)."""
    base = os.path.join(sysfs, "devices", "system", "node")
    try:
        nodes = sorted(int(d[4:]) for d in os.listdir(base) if d.startswith("node") and d[4:].isdigit())
        with open(os.path.join(base, f"node{node}", "distance")) as f:
            dist = [int(x) for x in f.read().split()]
    except (OSError, ValueError):
        return {}
    return {n: d for n, d in zip(nodes, dist)}


def p2p_caps(device: int = 0, sysfs: str = "/sys") -> dict:
    """CXL reachability of a GPU (the P2P caps CXL bit the fork declares but
    never sets, kern_bus_ctrl.c:769-774): per CXL node, the NUMA distance from the
    GPU's own node (the CPU-side hop a GPU<->CXL DMA crosses) and the nearest node."""
    info = lib.cxl_info()
    gnode = lib.device_numa_node(device) if device < lib.device_count() else -1
    dist = numa_distances(gnode, sysfs) if gnode >= 0 else {}
    cxl_dist = {n: dist.get(n, -1) for n in info["numa_nodes"]}
    reachable = [n for n, d in cxl_dist.items() if d >= 0]
    return {
        "cxl_supported": bool(info["memory_expander"]),
        "cxl_link_up": bool(info["link_up"]),
        "emulated": bool(info["emulated"]),
        "connectivity": "CXL" if info["memory_expander"] else "NONE",
        "gpu_numa_node": gnode,
        "cxl_numa_nodes": info["numa_nodes"],
        "cxl_numa_distance": cxl_dist,
        "nearest_cxl_node": min(reachable, key=lambda n: (cxl_dist[n], n)) if reachable else -1,
    }


def measure_bandwidth(device: int = 0, nbytes: int = 1 << 30, iters: int = 5, node: Optional[int] = None,
                      barrier=None) -> dict:
    """HBM<->CXL GB/s through the CXL ring (its configured engine: SDMA by default,
    one of the full-rate PCIe engines - tools/probe_cxl_paths.hip). Records the measured
    per-link bandwidth in the runtime's CXL info (replacing the fork's constant).
    ``barrier``: called before each timed direction, so that N processes (one per
    GPU) measure concurrently and the sum of their rates is the node aggregate."""
    import torch

    buf = CxlBuffer.allocate(nbytes, node=node if node is not None else (get_info()["numa_nodes"] or [None])[0])
    dst = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{device}")
    torch.cuda.synchronize()
    res = {}
    for name, d in (("cxl_to_gpu", DIR_CXL_TO_GPU), ("gpu_to_cxl", DIR_GPU_TO_CXL)):
        wait(buf.dma(dst.data_ptr(), device, 0, nbytes, d))
        if barrier is not None:
            barrier()
        t0 = time.perf_counter()
        tid = 0
        for _ in range(iters):
            tid = buf.dma(dst.data_ptr(), device, 0, nbytes, d)
        wait(tid)
        dt = time.perf_counter() - t0
        res[name + "_gbps"] = nbytes * iters / dt / 1e9
    lib.cxl_set_measured_bw(res["cxl_to_gpu_gbps"] * 1000.0)
    buf.unregister()
    res["emulated"] = get_info()["emulated"]
    return res
