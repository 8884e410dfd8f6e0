"""Device fault buffer + host fault-service thread (replayable-fault and
access-counter servicing, uvm_gpu_replayable_faults.c / uvm_gpu_access_counters.c /
uvm_gpu_isr.c analogs). Records are injected into the device-visible buffer the
way k_managed_gather writes them on a GPU."""
from __future__ import annotations

import ctypes
import time

import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20


class Rec(ctypes.Structure):
    _fields_ = [("range_id", ctypes.c_uint64), ("block", ctypes.c_uint32), ("page", ctypes.c_uint16),
                ("access", ctypes.c_uint8), ("kind", ctypes.c_uint8), ("proc", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


def _inject(records):
    put_addr, recs_addr, entries, _ = lib.fault_buffer_info(0)
    arr = (Rec * entries).from_address(recs_addr)
    for i, r in enumerate(records):
        arr[i] = r
    ctypes.c_uint32.from_address(put_addr).value = len(records)


def _wait(pred, timeout=10.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.01)
    return False


def test_fault_records_serviced_by_thread(fake_rt):
    assert ctypes.sizeof(Rec) == 24
    b = rt.malloc_managed(4 * MB, "faults")
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    lib.start_fault_service(100)
    _inject([Rec(b.id, 1, 7, 1, 0, 0, 0), Rec(b.id, 1, 7, 1, 0, 0, 0), Rec(b.id, 0, 3, 2, 0, 0, 0)])
    assert _wait(lambda: lib.fault_service_batches() >= 1)
    assert _wait(lambda: any(r["tier"] == "gpu" for r in b.residency(2 * MB)["resident_on"]))
    s = lib.stats()
    assert s["fault_batches"] >= 1 and s["faults_coalesced"] >= 1
    lib.stop_fault_service()
    b.free()


def test_access_counters_migrate_hot_block(fake_rt):
    lib.configure("perf_access_counter_threshold", 4)
    b = rt.malloc_managed(4 * MB, "hot")
    b.set_preferred_location("host:0")
    b.set_accessed_by(0)
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    # remote-access notifications (kind=1) for block 1 only
    _inject([Rec(b.id, 1, p, 1, 1, 0, 0) for p in range(4)])
    lib.poll_device_faults(0)
    s = lib.stats()
    assert s["access_counter_notifications"] == 4
    assert s["access_counter_migrations"] == 1
    assert any(r["tier"] == "gpu" for r in b.residency(2 * MB)["resident_on"])
    assert not any(r["tier"] == "gpu" for r in b.residency(0)["resident_on"])
    b.free()


def test_fault_buffer_overflow_is_counted(fake_rt):
    put_addr, _, entries, _ = lib.fault_buffer_info(0)
    ctypes.c_uint32.from_address(put_addr).value = entries + 10  # device wrote past the end
    from ogkm import tools

    q = tools.EventQueue(events=["FaultBufferOverflow"])
    lib.poll_device_faults(0)
    assert lib.fault_buffer_info(0)[3] == 10
    assert any(e["type"] == "FaultBufferOverflow" for e in q.read_dicts())
    q.close()
