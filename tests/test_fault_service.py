"""Device fault buffer + host fault-service thread (replayable-fault and
access-counter servicing, uvm_gpu_replayable_faults.c / uvm_gpu_access_counters.c /
uvm_gpu_isr.c analogs). Records are injected into the device-visible buffer the
way k_managed_gather writes them on a GPU."""
from __future__ import annotations

import ctypes
import time

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20


def _inject(records):
    """Append records with the device producer protocol (CAS on PUT, release-
    published sequence numbers): (range_id, block, page, access, kind, proc)."""
    assert lib.inject_device_faults(0, records) == len(records)


def _wait(pred, timeout=10.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.01)
    return False


def test_fault_records_serviced_by_thread(fake_rt):
    b = rt.malloc_managed(4 * MB, "faults")
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    lib.start_fault_service(100)
    _inject([(b.id, 1, 7, 1, 0, 0), (b.id, 1, 7, 1, 0, 0), (b.id, 0, 3, 2, 0, 0)])
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
    _inject([(b.id, 1, p, 1, 1, 0) for p in range(4)])
    lib.poll_device_faults(0)
    s = lib.stats()
    assert s["access_counter_notifications"] == 4
    assert s["access_counter_migrations"] == 1
    assert any(r["tier"] == "gpu" for r in b.residency(2 * MB)["resident_on"])
    assert not any(r["tier"] == "gpu" for r in b.residency(0)["resident_on"])
    b.free()


def test_fault_buffer_overflow_is_counted(fake_rt):
    info = lib.fault_buffer_info(0)
    n = info["entries"]
    b = rt.malloc_managed(2 * MB, "ov")
    from ogkm import tools

    q = tools.EventQueue(events=["FaultBufferOverflow"])
    # a full ring drops (and counts) what does not fit; nothing is overwritten
    assert lib.inject_device_faults(0, [(b.id, 0, p % 512, 1, 0, 0) for p in range(n + 10)]) == n
    lib.poll_device_faults(0)
    info = lib.fault_buffer_info(0)
    assert info["overflows"] == 10 and info["get"] == info["put"]
    assert any(e["type"] == "FaultBufferOverflow" for e in q.read_dicts())
    q.close()
    b.free()


def test_get_put_ring_concurrent_producers_lose_nothing(fake_rt):
    """Producers append while the host drains: every record arrives exactly
    once, in slot order per producer, across many wraps of the ring."""
    import threading

    n_prod, per = 4, 3 * lib.fault_buffer_info(0)["entries"]
    got = []
    stop = threading.Event()

    def drain():
        while not stop.is_set() or lib.fault_buffer_info(0)["put"] != lib.fault_buffer_info(0)["get"]:
            got.extend(lib.drain_fault_records(0))

    def produce(k):
        i = 0
        while i < per:
            if lib.inject_device_faults(0, [(99, k, i % 512, 1, 0, i)]):
                i += 1

    d = threading.Thread(target=drain)
    d.start()
    ps = [threading.Thread(target=produce, args=(k,)) for k in range(n_prod)]
    for t in ps:
        t.start()
    for t in ps:
        t.join()
    stop.set()
    d.join()
    assert len(got) == n_prod * per
    for k in range(n_prod):
        mine = [r[5] for r in got if r[1] == k]
        assert mine == list(range(per))


def test_replay_token_and_table_after_service(fake_rt):
    """A serviced batch bumps the replay token after its copies landed and the
    device residency table shows the block in HBM."""
    b = rt.malloc_managed(4 * MB, "rp")
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    table = lib.device_table(b.id)
    r0 = lib.fault_buffer_info(0)["replay"]
    _inject([(b.id, 1, 0xFFFF, 1, 0, 0)])  # whole block (what k_fault_gate records)
    lib.poll_device_faults(0)
    assert lib.fault_buffer_info(0)["replay"] == r0 + 1
    hbm = ctypes.c_uint64.from_address(table + 16).value
    assert hbm != 0
    assert lib.stats()["fault_replays"] >= 1
    b.free()


def test_access_counters_on_remote_leases_promote_hot_block(fake_rt):
    """Remote (zero-copy) leases are real GPU traffic to host memory: they feed
    the software access counters, and a block that crosses the threshold is
    migrated to the GPU on its next use instead of being mapped remotely."""
    lib.configure("perf_access_counter_threshold", 4)
    b = rt.malloc_managed(4 * MB, "remote-hot")
    b.set_preferred_location("host:0")
    b.set_accessed_by(0)
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    for _ in range(4):
        l = b.acquire(0, rt.READ)
        assert l.remote
        l.release()
    s = lib.stats()
    assert s["access_counter_notifications"] == 8            # 4 leases x 2 blocks
    l = b.acquire(0, rt.READ)
    assert not l.remote                                      # promoted: migrated to HBM
    l.release()
    assert lib.stats()["access_counter_migrations"] >= 2
    assert all(any(r["tier"] == "gpu" for r in b.residency(o)["resident_on"]) for o in (0, 2 * MB))
    b.free()


def test_user_channel_attribution_and_fatal_cancel(fake_rt):
    """Faults carry their channel (proc = dev | channel << 16, what the HIP
    producers record for a registered stream): per-channel counts, and a fault on
    a freed range is fatal for its channel only (uvm_user_channel.c +
    precise cancel, uvm_gpu_replayable_faults.c:2495-2875)."""
    b = rt.malloc_managed(4 * MB, "chan")
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    a_id = lib.register_channel(0, 0x1000, "decode")
    b_id = lib.register_channel(0, 0x2000, "prefill")
    assert lib.register_channel(0, 0x1000, "again") == a_id  # one channel per stream
    assert lib.fault_client(0, 0x1000) == a_id << 16 and lib.fault_client(0, 0x3000) == 0
    gone = rt.malloc_managed(2 * MB, "gone")
    gone_id = gone.id
    gone.free()
    _inject([(b.id, 0, 1, 1, 0, a_id << 16), (b.id, 1, 2, 1, 0, a_id << 16),
             (b.id, 1, 0, 1, 1, b_id << 16),          # remote access (access counter)
             (gone_id, 0, 0, 1, 0, b_id << 16)])      # fault on a freed range
    lib.poll_device_faults(0)
    ch = {c["name"]: c for c in lib.channels()}
    assert ch["decode"]["faults"] == 2 and ch["decode"]["error"] == "OK"
    assert ch["prefill"]["remote_accesses"] == 1 and ch["prefill"]["fatal_faults"] == 1
    assert ch["prefill"]["error"] != "OK"
    assert lib.global_status() == "OK"                 # the runtime carries on
    assert any(r["tier"] == "gpu" for r in b.residency(0)["resident_on"])
    lib.unregister_channel(b_id)
    assert [c["name"] for c in lib.channels()] == ["decode"]
    b.free()


def test_failed_service_cancels_channel_precisely(fake_rt):
    """A fault whose service fails (injected populate error) is cancelled for
    its channel only: the channel is marked errored, its cancel word is bumped
    before the replay token (a gate waiting on it exits with kGateCancelled),
    and a healthy channel's fault in the same batch is serviced
    (cancel_faults_precise, uvm_gpu_replayable_faults.c:2863)."""
    lib.init_device(0, 64 * MB)
    ok_buf = rt.malloc_managed(2 * MB, "ok")
    ok_buf.write(torch.ones(2 * MB, dtype=torch.uint8))
    bad = rt.malloc_managed(2 * MB, "bad")            # never written: its first fault must populate
    good_ch = lib.register_channel(0, 0x5000, "good")
    bad_ch = lib.register_channel(0, 0x6000, "bad")
    info0 = lib.fault_buffer_info(0)
    lib.inject("populate_error", 1)
    _inject([(bad.id, 0, 0xFFFF, 1, 0, bad_ch << 16)])
    lib.poll_device_faults(0)
    info1 = lib.fault_buffer_info(0)
    assert info1["cancel"][bad_ch % 64] == info0["cancel"][bad_ch % 64] + 1
    assert info1["cancel"][good_ch % 64] == info0["cancel"][good_ch % 64]
    assert info1["replay"] == info0["replay"] + 1     # the gate is woken, and sees the cancel
    ch = {c["name"]: c for c in lib.channels()}
    assert ch["bad"]["error"] != "OK" and ch["bad"]["cancelled_faults"] == 1
    assert ch["good"]["error"] == "OK"
    assert lib.stats()["faults_cancelled"] >= 1
    # the healthy channel's fault is serviced as usual, nothing cancelled
    _inject([(ok_buf.id, 0, 0xFFFF, 1, 0, good_ch << 16)])
    lib.poll_device_faults(0)
    info2 = lib.fault_buffer_info(0)
    assert info2["cancel"] == info1["cancel"] and info2["replay"] == info1["replay"] + 1
    assert any(r["tier"] == "gpu" for r in ok_buf.residency(0)["resident_on"])
    assert lib.global_status() == "OK"
    lib.unregister_channel(good_ch)
    lib.unregister_channel(bad_ch)
    bad.free()
    ok_buf.free()


def test_channel_ids_never_share_a_cancel_word(fake_rt):
    """Channel ids stay below the 64 cancel words (no aliasing: channel 64 would
    otherwise cancel the gates of unattributed kernels), and a failed fault of
    an unattributed stream (channel 0) bumps no cancel word at all - its gate
    falls back to the replay / timeout path."""
    live = [lib.register_channel(0, 0x10000 + i, f"c{i}") for i in range(63)]
    assert len(set(live)) == 63 and max(live) == 63
    with pytest.raises(Exception, match="no channel slot left"):
        lib.register_channel(0, 0x20000, "one too many")
    for i in live:
        lib.unregister_channel(i)
    lib.init_device(0, 64 * MB)
    bad = rt.malloc_managed(2 * MB, "bad0")
    info0 = lib.fault_buffer_info(0)
    lib.inject("populate_error", 1)
    _inject([(bad.id, 0, 0xFFFF, 1, 0, 0)])  # no channel
    lib.poll_device_faults(0)
    info1 = lib.fault_buffer_info(0)
    assert info1["cancel"] == info0["cancel"]
    assert info1["replay"] == info0["replay"] + 1
    bad.free()
