"""Software access counters fed by local-copy leases (reference
uvm_gpu_access_counters.c:40-84, :1617 service_notifications): a block whose
policy keeps it remote (preferred host + accessed_by the GPU) but whose
consumer needs it at its own device address - the transparent mode's op holds
(acquire allow_remote=False) - is served by a local duplicate each time, and
every such access is counted; at perf_access_counter_threshold the block is
promoted and its next access migrates it to the GPU (no more duplicates)."""
from __future__ import annotations

import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20


def _remote_tensor():
    lib.init_device(0, 32 * MB)
    b = rt.malloc_managed(4 * MB, "remote", cpu_view=False)
    b.set_preferred_location(rt.Loc.host(lib.host_node()))
    b.set_accessed_by(0)
    b.write(torch.arange(MB, dtype=torch.int32))
    return b


def test_local_copy_leases_feed_access_counters_and_promote(fake_rt):
    lib.configure("perf_access_counter_threshold", 8)
    b = _remote_tensor()
    lib.reset_counters()
    for i in range(7):
        lease = b.acquire(0, rt.READ, allow_remote=False)
        lease.wait(0)
        lease.release(0)
        b.evict("gpu:0")  # the duplicate is dropped again: the next access is another remote access
    s = lib.stats()
    assert s["remote_fallbacks"] == 7 * 2 and s["access_counter_notifications"] == 7 * 2, s  # 2 blocks each
    assert s["access_counter_migrations"] == 0
    lease = b.acquire(0, rt.READ, allow_remote=False)  # the 8th access reaches the threshold
    lease.wait(0)
    lease.release(0)
    b.evict("gpu:0")
    lease = b.acquire(0, rt.READ, allow_remote=False)  # promoted: migrated, not duplicated
    lease.wait(0)
    s = lib.stats()
    assert s["access_counter_migrations"] >= 2, s
    assert s["remote_fallbacks"] == 8 * 2, s  # the promoted access was not a remote decision
    assert not lease.remote
    lease.release(0)
    assert torch.equal(b.read().view(torch.int32), torch.arange(MB, dtype=torch.int32))


def test_remote_leases_stay_zero_copy_below_threshold(fake_rt):
    """With allow_remote (the engine's embedding path) the same block is read in
    place - a remote lease, no copy - and counted the same way."""
    lib.configure("perf_access_counter_threshold", 1000)
    b = _remote_tensor()
    lib.reset_counters()
    for _ in range(5):
        lease = b.acquire(0, rt.READ)
        lease.wait(0)
        assert lease.remote
        lease.release(0)
    s = lib.stats()
    assert s["bytes_xfer_htd"] == 0 and s["access_counter_notifications"] == 10, s
