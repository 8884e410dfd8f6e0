"""GPU tests of the device fault path on a real MI355X: the GET/PUT fault ring
under a kernel that appends while the host drains, and the fault gate
(replayable-fault stall -> host service -> replay -> the kernel behind the gate
reads the migrated data through the device residency table).

Reference behaviour: uvm_gpu_replayable_faults.c:558 (GET write-back), :844-988
(fetch: a record is consumed only once valid), :2906 (batch service), :2986-3022
(replay after the batch).
"""
from __future__ import annotations

import threading
import time

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

pytestmark = pytest.mark.gpu

MB = 1 << 20


def test_fault_ring_kernel_appends_while_host_drains(gpu_rt):
    """64 waves append 64 records per lane (256 Ki records, 64 wraps of a 4 Ki
    ring) while a host thread drains: every record arrives exactly once (the
    producers wait for ring space instead of dropping)."""
    waves, per_lane = 64, 64
    total = waves * 64 * per_lane
    entries = lib.fault_buffer_info(0)["entries"]
    assert total >= 16 * entries
    gave_up = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    got = []
    t_end = time.time() + 60

    def drain():
        while len(got) < total and time.time() < t_end:
            got.extend(lib.drain_fault_records(0, 1 << 16))

    d = threading.Thread(target=drain)
    d.start()
    lib.fault_stress(0, waves, per_lane, gave_up.data_ptr(), s.cuda_stream)
    d.join()
    s.synchronize()
    assert int(gave_up) == 0
    assert len(got) == total, (len(got), total)
    ids = torch.tensor([(r[1] << 8) | r[2] for r in got], dtype=torch.int64)
    assert torch.equal(torch.sort(ids).values, torch.sort(
        (torch.arange(waves * 64).repeat_interleave(per_lane) << 8) | torch.arange(per_lane).repeat(waves * 64)).values)
    assert all(r[5] == r[1] for r in got[:1000])   # proc field = producer lane id
    assert lib.fault_buffer_info(0)["overflows"] == 0


def test_fault_gate_stalls_until_serviced_then_fetch_reads_hbm(gpu_rt):
    n = 8 * MB
    ref = torch.randint(0, 1 << 30, (n // 4,), dtype=torch.int32)
    b = rt.malloc_managed(n, "gate")
    b.write(ref)
    assert b.residency(0)["resident_on"][0]["tier"] == "host"
    lib.device_table(b.id)
    s = torch.cuda.Stream()
    lib.register_table_stream(0, s.cuda_stream)
    status = torch.full((2,), 7, dtype=torch.int32, device="cuda")
    out = torch.zeros(n // 4, dtype=torch.int32, device="cuda")
    lib.start_fault_service(50)
    try:
        lib.fault_gate(b.id, 0, n, 0, s.cuda_stream, status.data_ptr(), timeout_ms=10000)
        lib.table_fetch(b.id, 0, n, out.data_ptr(), 0, s.cuda_stream)
        s.synchronize()
    finally:
        lib.stop_fault_service()
        lib.register_table_stream(0, s.cuda_stream, False)
    st = status.cpu().tolist()
    assert st[0] == 0 and st[1] >= 1, st      # resolved after at least one replay
    assert torch.equal(out.cpu(), ref)
    assert all(any(r["tier"] == "gpu" for r in b.residency(o)["resident_on"]) for o in range(0, n, 2 * MB))
    stats = lib.stats()
    assert stats["fault_replays"] >= 1 and stats["gpu_page_faults"] >= 4
    b.free()


def test_fault_gate_times_out_without_service(gpu_rt):
    b = rt.malloc_managed(2 * MB, "nogate")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    lib.device_table(b.id)
    status = torch.full((2,), 7, dtype=torch.int32, device="cuda")
    t0 = time.perf_counter()
    lib.fault_gate(b.id, 0, 2 * MB, 0, torch.cuda.current_stream().cuda_stream, status.data_ptr(), timeout_ms=50)
    torch.cuda.synchronize()
    assert status.cpu().tolist()[0] == 2            # cancelled, and the kernel exited
    assert time.perf_counter() - t0 < 5
    lib.drain_fault_records(0)                       # the recorded faults are not serviced here
    b.free()


def test_fault_gate_cancelled_when_service_fails(gpu_rt):
    """Precise cancel on hardware: the gate's fault cannot be serviced (one
    injected populate error), so the host cancels the gate's channel within one
    poll - the gate exits with kGateCancelled (3) instead of re-recording until
    its timeout, and the channel reports an error."""
    b = rt.malloc_managed(2 * MB, "cancel")           # never written: the fault must populate
    lib.device_table(b.id)
    s = torch.cuda.Stream()
    ch = lib.register_channel(0, s.cuda_stream, "gated")
    status = torch.full((2,), 7, dtype=torch.int32, device="cuda")
    lib.inject("populate_error", 1)
    t0 = time.perf_counter()
    lib.fault_gate(b.id, 0, 2 * MB, 0, s.cuda_stream, status.data_ptr(), timeout_ms=20000)
    polls = 0
    while not s.query() and time.perf_counter() - t0 < 15:
        polls += lib.poll_device_faults(0) > 0
        time.sleep(0.001)
    s.synchronize()
    dt = time.perf_counter() - t0
    st = status.cpu().tolist()
    chans = {c["id"]: c for c in lib.channels()}
    lib.unregister_channel(ch)
    assert st[0] == 3, st                             # cancelled, not resolved / timed out
    assert 1 <= polls <= 2 and dt < 5, (polls, dt)  # a 1 ms re-record may race the first service
    assert chans[ch]["error"] != "OK" and chans[ch]["cancelled_faults"] == 1, chans[ch]
    b.free()


def test_table_shootdown_fences_queued_readers(gpu_rt):
    """Evicting a block listed in a device table clears its entry and fences
    the chunk on the registered table streams (no stale-chunk reads)."""
    lib.init_device(0, 16 * MB)
    n = 8 * MB
    ref = torch.randint(0, 1 << 30, (n // 4,), dtype=torch.int32)
    b = rt.malloc_managed(n, "sd")
    b.write(ref)
    b.migrate("gpu:0")
    lib.device_table(b.id)
    s = torch.cuda.Stream()
    lib.register_table_stream(0, s.cuda_stream)
    out = torch.zeros(n // 4, dtype=torch.int32, device="cuda")
    lib.table_fetch(b.id, 0, n, out.data_ptr(), 0, s.cuda_stream)
    other = rt.malloc_managed(16 * MB, "pressure")
    other.fill(0x55555555)
    other.migrate("gpu:0")                           # evicts b's chunks while the fetch may be queued
    s.synchronize()
    lib.register_table_stream(0, s.cuda_stream, False)
    assert torch.equal(out.cpu(), ref)
    assert lib.stats()["table_shootdowns"] >= 1
    other.free()
    b.free()
