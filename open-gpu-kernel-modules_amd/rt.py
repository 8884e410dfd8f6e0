"""Public runtime API: managed memory with cudaMallocManaged / cudaMemAdvise /
cudaMemPrefetchAsync-*shaped* calls in our own namespace (no CUDA shims).

Reference parity (user contract of the UVM driver, kernel-open/nvidia-uvm/uvm.h):
  malloc_managed        <- UvmMemMap / mmap of /dev/nvidia-uvm          (uvm.c:792)
  mem_advise            <- UvmSetPreferredLocation / SetAccessedBy /
                           EnableReadDuplication                         (uvm.h:2276,2457,2615)
  mem_prefetch_async    <- UvmMigrate(Async)                              (uvm_migrate.c:882)
  residency_info        <- UVM_TEST_VA_RESIDENCY_INFO                     (uvm_test_ioctl.h:626-674)
  range groups          <- UvmCreateRangeGroup / PreventMigration        (uvm_range_group.c:88)
  map_external          <- UvmMapExternalAllocation                       (uvm_map_external.c:1093)
  alloc_device_p2p      <- UvmAllocDeviceP2P                              (uvm_va_range_device_p2p.c:499)

MI355X-native semantics: there are no hardware replayable faults (no XNACK), so a
GPU "fault" is raised in software at tensor granularity by :meth:`ManagedBuffer.acquire`
(or recorded by our own HIP kernels, see ``ops.managed_gather``); the CPU side uses
real page faults on the buffer's CPU view (SIGSEGV handled in the native core).
"""
from __future__ import annotations

import contextlib
import dataclasses
from typing import Iterable, Optional

from ._native import RuntimeStatusError, lib

__all__ = [
    "Loc", "init", "shutdown", "is_initialized", "configure", "get_config", "malloc_managed", "ManagedBuffer",
    "Lease", "mem_advise", "mem_prefetch_async", "mem_range_get_attribute", "stats", "sync", "RuntimeStatusError",
    "ADVISE_SET_READ_MOSTLY", "ADVISE_UNSET_READ_MOSTLY", "ADVISE_SET_PREFERRED_LOCATION",
    "ADVISE_UNSET_PREFERRED_LOCATION", "ADVISE_SET_ACCESSED_BY", "ADVISE_UNSET_ACCESSED_BY", "CPU",
    "READ", "WRITE", "ATOMIC", "PREFETCH", "create_range_group", "map_external", "alloc_device_p2p",
]

ADVISE_SET_READ_MOSTLY = 1
ADVISE_UNSET_READ_MOSTLY = 2
ADVISE_SET_PREFERRED_LOCATION = 3
ADVISE_UNSET_PREFERRED_LOCATION = 4
ADVISE_SET_ACCESSED_BY = 5
ADVISE_UNSET_ACCESSED_BY = 6

READ, WRITE, ATOMIC, PREFETCH = 1, 2, 3, 4
CPU = 32  # processor id of the CPU (GPUs are 0..31)

RANGE_STABLE_VA = 1
RANGE_NO_CPU_VIEW = 2
RANGE_PACKED_BF16 = 4

_TIERS = {"gpu": 0, "hbm": 0, "host": 1, "cpu": 1, "cxl": 2}


@dataclasses.dataclass(frozen=True)
class Loc:
    """A memory location: ``gpu:i`` (HBM of GPU i), ``host:n`` (DRAM of NUMA node n)
    or ``cxl:n`` (CXL.mem NUMA node n)."""

    tier: str
    id: int = 0

    @staticmethod
    def gpu(i: int = 0) -> "Loc":
        return Loc("gpu", i)

    @staticmethod
    def host(n: Optional[int] = None) -> "Loc":
        return Loc("host", lib.host_node() if n is None else n)

    @staticmethod
    def cxl(n: Optional[int] = None) -> "Loc":
        if n is None:
            nodes = lib.cxl_info()["numa_nodes"]
            if not nodes:
                raise RuntimeStatusError("no CXL memory node (set cxl_emulate_node to emulate one)")
            n = lib.cxl_nearest_node(lib.host_node())  # the pool nearest this runtime's host node
        return Loc("cxl", n)

    @staticmethod
    def parse(s: "str | Loc") -> "Loc":
        if isinstance(s, Loc):
            return s
        t, _, i = str(s).partition(":")
        t = t.lower()
        if t in ("host", "cpu") and not i:
            return Loc.host()
        if t == "cxl" and not i:
            return Loc.cxl()
        return Loc("gpu" if t == "hbm" else ("host" if t == "cpu" else t), int(i or 0))

    @property
    def code(self) -> tuple[int, int]:
        return _TIERS[self.tier], self.id

    def __str__(self) -> str:
        return f"{self.tier}:{self.id}"


# --------------------------------------------------------------------------- lifecycle
def init(backend: str = "auto", fake_devices: int = 2, fake_hbm_mb: int = 256, hbm_budget: Optional[dict] = None,
         **config) -> str:
    """Bring the runtime up. ``backend`` is ``auto`` | ``hip`` | ``fake`` (CPU-only
    devices). ``hbm_budget`` maps GPU id -> arena bytes (the oversubscription cap).
    Extra keyword arguments are config knobs (same names as the reference's UVM
    module parameters, see ``config_names()``)."""
    for k, v in config.items():
        lib.configure(k, int(v))
    name = lib.init(backend, fake_devices, fake_hbm_mb)
    for k, v in config.items():
        lib.configure(k, int(v))
    for dev, nbytes in (hbm_budget or {}).items():
        lib.init_device(int(dev), int(nbytes))
    return name


def shutdown() -> None:
    lib.shutdown()


def is_initialized() -> bool:
    return lib.is_initialized()


def configure(**kw) -> None:
    for k, v in kw.items():
        lib.configure(k, int(v))


def get_config(name: str) -> int:
    return lib.get_config(name)


def config_names() -> list[str]:
    return list(lib.config_names())


def device_count() -> int:
    return lib.device_count()


def backend() -> str:
    return lib.backend_name()


def sync() -> None:
    lib.sync_all()


def stats() -> dict:
    return lib.stats()


# --------------------------------------------------------------------------- dtype helpers
def _dl_dtype(dtype):
    import torch

    table = {
        torch.float32: (2, 32), torch.float16: (2, 16), torch.bfloat16: (4, 16), torch.float64: (2, 64),
        torch.int8: (0, 8), torch.uint8: (1, 8), torch.int16: (0, 16), torch.int32: (0, 32), torch.int64: (0, 64),
    }
    if dtype not in table:
        raise TypeError(f"unsupported dtype {dtype}")
    return table[dtype]


def _tensor_from_ptr(ptr: int, shape, dtype, device: str, device_id: int = 0, range_id: int = 0):
    import torch

    code, bits = _dl_dtype(dtype)
    dev_type = 10 if device == "cuda" else 1  # kDLROCM / kDLCPU
    cap = lib.dlpack(ptr, [int(s) for s in shape], code, bits, dev_type, device_id, range_id)
    return torch.utils.dlpack.from_dlpack(cap)


def current_stream_handle(device: int = 0) -> int:
    import torch

    if lib.backend_name() == "fake" or not torch.cuda.is_available():
        return 0
    return int(torch.cuda.current_stream(device).cuda_stream)


# --------------------------------------------------------------------------- leases
class Lease:
    """A software-fault service result: [offset, offset+nbytes) of a managed buffer
    is resident (or remotely mapped) for processor ``proc`` at ``dptr`` until
    released. GPU consumers must ``wait(stream)`` (a GPU-side dependency on the
    migration ring) before use and ``release(stream)`` after their last use."""

    def __init__(self, buf: "ManagedBuffer", info: dict, proc: int, offset: int, nbytes: int):
        self.buf = buf
        self.id = info["id"]
        self.dptr = info["dptr"]
        self.remote = info["remote"]
        self.proc = proc
        self.offset = offset
        self.nbytes = nbytes
        self._released = False

    def wait(self, stream: Optional[int] = None) -> None:
        """Make the lease's data usable. ``stream=None``: the current stream of the
        lease's GPU waits for the migration GPU-side (the host does not block,
        also when that is the null stream); ``stream=<handle>``: that stream
        waits; ``stream=0``: the host waits (CPU leases, fake backend, tests)."""
        if self.proc == CPU or lib.backend_name() == "fake":
            lib.lease_wait(self.id, 0, False)
        elif stream is None:
            lib.lease_wait(self.id, current_stream_handle(self.proc), True)
        else:
            lib.lease_wait(self.id, int(stream), bool(stream))

    def wait_host(self) -> None:
        lib.lease_wait(self.id, 0, False)

    def tensor(self, shape, dtype):
        dev = "cpu" if self.proc == CPU or lib.backend_name() == "fake" else "cuda"
        return _tensor_from_ptr(self.dptr, shape, dtype, dev, 0 if self.proc == CPU else self.proc, self.buf.id)

    def release(self, stream: Optional[int] = None) -> None:
        if self._released:
            return
        lib.release(self.id, current_stream_handle(self.proc) if stream is None and self.proc != CPU else (stream or 0))
        self._released = True

    def __enter__(self):
        self.wait()
        return self

    def __exit__(self, *a):
        self.release()

    def __del__(self):
        try:
            if not self._released and lib.is_initialized():
                self.release(0)
        except Exception:
            pass


# --------------------------------------------------------------------------- managed buffers
# Callables run with the buffer just before a range is freed (see p2p.py).
_free_hooks: list = []


class ManagedBuffer:
    """A managed allocation (one VA range of 2 MB blocks)."""

    def __init__(self, rid: int):
        self.id = rid
        info = lib.range_info(rid)
        self.size = info["size"]
        self.addr = info["addr"]          # CPU view (the canonical pointer)
        self.dev_va = info["dev_va"]      # stable device VA (RANGE_STABLE_VA only)
        self.name = info["name"]
        self._freed = False

    # -- policy
    def advise(self, advice: int, loc: "str | Loc | None" = None, offset: int = 0, length: Optional[int] = None,
               proc: Optional[int] = None) -> None:
        length = self.size - offset if length is None else length
        t, i = Loc.parse(loc).code if loc is not None else (0, 0)
        lib.mem_advise(self.id, offset, length, advice, t, i, CPU if proc is None else proc)

    def set_preferred_location(self, loc, offset: int = 0, length: Optional[int] = None):
        self.advise(ADVISE_SET_PREFERRED_LOCATION, loc, offset, length)

    def set_read_mostly(self, on: bool = True, offset: int = 0, length: Optional[int] = None):
        self.advise(ADVISE_SET_READ_MOSTLY if on else ADVISE_UNSET_READ_MOSTLY, None, offset, length)

    def set_accessed_by(self, proc: int, on: bool = True, offset: int = 0, length: Optional[int] = None):
        self.advise(ADVISE_SET_ACCESSED_BY if on else ADVISE_UNSET_ACCESSED_BY, None, offset, length, proc)

    # -- migration
    def prefetch(self, loc, offset: int = 0, length: Optional[int] = None, needed_at: int = 0):
        """``needed_at`` (op clock, next-use mode): evict only data needed later,
        or raise (NO_MEMORY) and leave the data where it is."""
        length = self.size - offset if length is None else length
        t, i = Loc.parse(loc).code
        return lib.prefetch(self.id, offset, length, t, i, int(needed_at))

    def resident_bytes(self, loc, offset: int = 0, length: Optional[int] = None) -> int:
        """Bytes of [offset, offset + length) resident at ``loc`` (page granular)."""
        length = self.size - offset if length is None else length
        t, i = Loc.parse(loc).code
        return lib.resident_bytes(self.id, t, i, offset, length)

    def hint_next_use(self, when: int) -> None:
        """Op-clock time of this range's next use: its HBM chunks are then evicted
        in next-use (Belady) order - see lib.set_op_clock."""
        lib.hint_next_use(self.id, int(when))

    def migrate(self, loc, offset: int = 0, length: Optional[int] = None) -> None:
        length = self.size - offset if length is None else length
        t, i = Loc.parse(loc).code
        lib.migrate(self.id, offset, length, t, i)

    def evict(self, loc) -> None:
        t, i = Loc.parse(loc).code
        lib.evict(self.id, t, i)

    # -- software faults
    def acquire(self, proc: int = 0, access: int = READ, offset: int = 0, length: Optional[int] = None,
                allow_remote: bool = True) -> Lease:
        length = self.size - offset if length is None else length
        return Lease(self, lib.acquire(self.id, offset, length, proc, access, allow_remote), proc, offset, length)

    # -- data
    def write(self, data, offset: int = 0) -> None:
        """Copy a torch tensor / bytes-like object into the buffer."""
        import torch

        if isinstance(data, torch.Tensor):
            t = data.contiguous()
            dev = t.device.index if t.is_cuda else -1
            if t.is_cuda:
                torch.cuda.current_stream(t.device).synchronize()
            lib.write(self.id, offset, t.data_ptr(), t.numel() * t.element_size(), dev if dev is not None else 0)
        else:
            mv = memoryview(data).cast("B")
            import ctypes

            buf = (ctypes.c_char * len(mv)).from_buffer_copy(mv)
            lib.write(self.id, offset, ctypes.addressof(buf), len(mv), -1)

    def read(self, out=None, offset: int = 0, nbytes: Optional[int] = None):
        import torch

        if out is None:
            nbytes = self.size - offset if nbytes is None else nbytes
            out = torch.empty(nbytes, dtype=torch.uint8)
        t = out
        dev = t.device.index if t.is_cuda else -1
        lib.read(self.id, offset, t.data_ptr(), t.numel() * t.element_size(), dev if dev is not None else 0)
        return out

    def fill(self, pattern: int, offset: int = 0, nbytes: Optional[int] = None) -> None:
        lib.fill(self.id, offset, self.size - offset if nbytes is None else nbytes, pattern & 0xFFFFFFFF)

    def cpu_view(self, dtype=None, shape=None):
        """Torch CPU tensor aliasing the CPU view: touching it raises real CPU page
        faults that migrate data to the host (the UVM CPU-fault path)."""
        import torch

        dtype = dtype or torch.uint8
        esz = torch.empty((), dtype=dtype).element_size()
        shape = shape or (self.size // esz,)
        return _tensor_from_ptr(self.addr, shape, dtype, "cpu", 0, self.id)

    def residency(self, offset: int = 0) -> dict:
        return lib.residency_info(self.id, offset)

    def set_range_group(self, group: int) -> None:
        lib.set_range_group(self.id, group)

    def free(self) -> None:
        if not self._freed:
            # Importers of this memory (p2p regions) are told first, so their
            # pins are dropped before the range goes away (peermem free callback).
            for hook in list(_free_hooks):
                hook(self)
            lib.free(self.id)
            self._freed = True

    def __repr__(self) -> str:
        return f"ManagedBuffer(id={self.id}, size={self.size}, addr={self.addr:#x}, name={self.name!r})"


def malloc_managed(nbytes: int, name: str = "", stable_va: bool = False, device: int = 0,
                   cpu_view: bool = True, packed_bf16: bool = False) -> ManagedBuffer:
    """``packed_bf16``: the contents are bf16 and read-only on GPUs; host / CXL
    copies are stored BF12-packed (lossless, ~0.75x) and decoded by the H2D copy
    kernel, cutting PCIe bytes for streamed weights. Implies no CPU view."""
    flags = ((RANGE_STABLE_VA if stable_va else 0) | (0 if cpu_view else RANGE_NO_CPU_VIEW)
             | (RANGE_PACKED_BF16 if packed_bf16 else 0))
    return ManagedBuffer(lib.malloc_managed(int(nbytes), flags, name, device))


def map_external(ptr: int, nbytes: int, device: int, name: str = "") -> ManagedBuffer:
    return ManagedBuffer(lib.map_external(ptr, nbytes, device, name))


def alloc_device_p2p(nbytes: int, device: int, name: str = "") -> ManagedBuffer:
    return ManagedBuffer(lib.alloc_device_p2p(nbytes, device, name))


def mem_advise(buf: ManagedBuffer, advice: int, loc=None, offset: int = 0, length: Optional[int] = None,
               proc: Optional[int] = None) -> None:
    buf.advise(advice, loc, offset, length, proc)


def mem_prefetch_async(buf: ManagedBuffer, loc, offset: int = 0, length: Optional[int] = None, stream=None):
    """Queue the migration on the io_uring-style ring; returns a Tracker. If
    ``stream`` is given, the stream waits (GPU-side) for the migration."""
    tr = buf.prefetch(loc, offset, length)
    if stream is not None:
        tr.gpu_wait(int(stream))
    return tr


def mem_range_get_attribute(buf: ManagedBuffer, attribute: str, offset: int = 0):
    info = buf.residency(offset)
    if attribute == "read_mostly":
        return info["read_mostly"]
    if attribute == "preferred_location":
        p = info["preferred"]
        return None if p is None else Loc(p["tier"], p["id"])
    if attribute == "accessed_by":
        m = info["accessed_by"]
        return [i for i in range(64) if (m >> i) & 1]
    if attribute == "last_prefetch_location":
        r = info["resident_on"]
        return None if not r else Loc(r[-1]["tier"], r[-1]["id"])
    raise KeyError(attribute)


def create_range_group(migratable: bool = True) -> int:
    g = lib.create_range_group()
    lib.set_group_migratable(g, migratable)
    return g


def set_range_group_migratable(group: int, migratable: bool) -> None:
    lib.set_group_migratable(group, migratable)


@contextlib.contextmanager
def acquired(bufs: Iterable[ManagedBuffer], proc: int = 0, access: int = READ):
    leases = [b.acquire(proc, access) for b in bufs]
    try:
        for l in leases:
            l.wait()
        yield leases
    finally:
        for l in leases:
            l.release()
