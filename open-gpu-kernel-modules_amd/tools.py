"""Tools event queues and counters (analog of the UVM tools API:
UvmToolsCreateEventQueue uvm.h:3588, event types uvm_types.h:362-392, counters
uvm_types.h:283-313, queue protocol uvm_tools.c:448-509).

Events are 64-byte records produced by the native core into an mmap'ed
single-producer ring (optionally in /dev/shm for out-of-process readers).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ._native import lib

EVENT_TYPES = {
    1: "CpuFault", 2: "Migration", 3: "GpuFault", 4: "GpuFaultReplay", 5: "FaultBufferOverflow", 6: "FatalFault",
    7: "ReadDuplicate", 8: "ReadDuplicateInvalidate", 9: "PageSizeChange", 10: "ThrashingDetected",
    11: "ThrottlingStart", 12: "ThrottlingEnd", 13: "MapRemote", 14: "Eviction", 15: "Prefetch",
    16: "AccessCounter", 17: "CxlDma", 18: "RingError", 19: "Checkpoint",
}
EVENT_IDS = {v: k for k, v in EVENT_TYPES.items()}
CAUSES = ["User", "Coherence", "Prefetch", "Eviction", "AccessCounters", "ApiMigrate", "Thrashing", "Cxl"]

EVENT_DTYPE = np.dtype([
    ("type", "u1"), ("cause", "u1"), ("src_slot", "u1"), ("dst_slot", "u1"), ("processor", "<u4"),
    ("address", "<u8"), ("bytes", "<u8"), ("ts_begin_ns", "<u8"), ("ts_end_ns", "<u8"), ("range_id", "<u8"),
    ("seq", "<u8"), ("aux", "<u8"),
])
assert EVENT_DTYPE.itemsize == 64


def slot_name(slot: int) -> str:
    return f"gpu:{slot}" if slot < 32 else f"node:{slot - 32}"


class EventQueue:
    """A tools event queue. ``events`` is a list of names (default: all)."""

    def __init__(self, entries: int = 4096, events: Optional[list[str]] = None, shm_name: str = ""):
        mask = 0xFFFFFFFF if events is None else sum(1 << EVENT_IDS[e] for e in events)
        self.qid = lib.tools_create_queue(entries, mask, shm_name)

    def read(self, max_events: int = 65536) -> np.ndarray:
        raw = lib.tools_read(self.qid, max_events)
        return np.frombuffer(raw, dtype=EVENT_DTYPE).copy()

    def read_dicts(self, max_events: int = 65536) -> list[dict]:
        out = []
        for e in self.read(max_events):
            out.append({
                "type": EVENT_TYPES.get(int(e["type"]), str(e["type"])),
                "cause": CAUSES[int(e["cause"])] if int(e["cause"]) < len(CAUSES) else int(e["cause"]),
                "src": slot_name(int(e["src_slot"])), "dst": slot_name(int(e["dst_slot"])),
                "processor": int(e["processor"]), "address": int(e["address"]), "bytes": int(e["bytes"]),
                "range_id": int(e["range_id"]), "ts_begin_ns": int(e["ts_begin_ns"]), "seq": int(e["seq"]),
            })
        return out

    def dropped(self) -> dict:
        d = lib.tools_dropped(self.qid)
        return {EVENT_TYPES.get(i, str(i)): n for i, n in enumerate(d) if n}

    def close(self) -> None:
        if self.qid is not None:
            lib.tools_destroy_queue(self.qid)
            self.qid = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def counters() -> dict:
    s = lib.stats()
    return {k: s[k] for k in lib.counter_names()}


def reset_counters() -> None:
    lib.reset_counters()


def prometheus_text(prefix: str = "ogkm") -> str:
    """Counters + arena gauges in Prometheus text exposition format (procfs analog)."""
    s = lib.stats()
    lines = []
    for k in lib.counter_names():
        lines.append(f"# TYPE {prefix}_{k} counter")
        lines.append(f"{prefix}_{k} {s[k]}")
    for a in s["arenas"]:
        for key in ("capacity", "allocated", "peak", "pinned", "evictions"):
            lines.append(f'{prefix}_arena_{key}{{arena="{a["name"]}"}} {a[key]}')
    lines.append(f"{prefix}_lock_violations {s['lock_violations']}")
    return "\n".join(lines) + "\n"


def read_process_memory(addr: int, nbytes: int) -> bytes:
    """Read managed memory at a virtual address wherever its valid copy lives
    (UVM_TOOLS_READ_PROCESS_MEMORY, uvm_tools.c:2591)."""
    return lib.tools_read_process_memory(addr, nbytes)


def write_process_memory(addr: int, data: bytes) -> None:
    """Write managed memory at a virtual address (UVM_TOOLS_WRITE_PROCESS_MEMORY,
    uvm_tools.c:2601); other copies of the written pages are invalidated."""
    lib.tools_write_process_memory(addr, bytes(data))


class trace_range:
    """``with tools.trace_range("step"):`` - a roctx range around Python code
    (shown by ``rocprofv3 --marker-trace``); the runtime wraps its own fault
    batches, migrations, evictions and leases the same way (config trace_ranges)."""

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        lib.range_push(self.name)
        return self

    def __exit__(self, *exc):
        lib.range_pop()
        return False
