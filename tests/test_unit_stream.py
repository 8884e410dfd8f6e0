"""Native per-unit protocol (csrc/core/unit_stream.cpp) on the fake backend:
the streamed path (window prefetch, next-use hints) and hold mode - after a
pass with no eviction and no streaming, released units keep their leases until
their next use; the first eviction somebody else causes ends it."""
from __future__ import annotations

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20


def _units(n, mb):
    bufs = []
    for i in range(n):
        b = rt.malloc_managed(mb * MB, f"u{i}")
        b.write(torch.full((mb * MB,), i + 1, dtype=torch.uint8))
        bufs.append(b)
    return bufs


def _pass(us, bufs, stream, check=True):
    for p, b in enumerate(bufs):
        lid, dptr = us.use(p, stream)
        if check:
            lib.debug_stream_sync(stream)
            t = rt._tensor_from_ptr(dptr, (4096,), torch.uint8, "cpu", 0, b.id)
            assert int(t[0]) == p + 1 and int(t[-1]) == p + 1
        us.release(lid, stream)


def test_hold_mode_when_everything_fits(fake_rt):
    lib.init_device(0, 48 * MB)  # 24 chunks: 4 units x 8 MB fit
    bufs = _units(4, 8)
    s = lib.debug_stream_create(0)
    us = lib.UnitStream(0, [b.id for b in bufs], 16 * MB, True, 2)
    for _ in range(4):
        _pass(us, bufs, s)
    st = us.stats()
    assert st["held"] >= 4, st  # pass 4 reused pass 3's leases
    assert st["hold_drops"] == 0, st
    # someone else needs HBM: an eviction ends hold mode at the next use
    other = rt.malloc_managed(40 * MB, "other")
    other.write(torch.zeros(40 * MB, dtype=torch.uint8))
    l = other.acquire(0, rt.WRITE)
    l.wait(0)
    l.release(0)
    _pass(us, bufs, s)
    assert us.stats()["hold_drops"] >= 1
    lib.debug_stream_sync(s)
    del us
    lib.debug_stream_destroy(s)
    for b in bufs + [other]:
        b.free()


def test_no_hold_under_oversubscription(fake_rt):
    lib.init_device(0, 24 * MB)  # 12 chunks: 4 units x 8 MB stream
    bufs = _units(4, 8)
    s = lib.debug_stream_create(0)
    us = lib.UnitStream(0, [b.id for b in bufs], 8 * MB, True, 2)
    for _ in range(4):
        _pass(us, bufs, s)
    assert us.stats()["held"] == 0
    lib.debug_stream_sync(s)
    del us
    lib.debug_stream_destroy(s)
    for b in bufs:
        b.free()


def test_write_to_held_unit_is_not_refused(fake_rt):
    """Hold mode keeps a lease on every unit between passes; a weight update
    between decode steps (a CPU write to a held unit) must still go through -
    the held leases are soft pins, let go on demand - and the next pass sees
    the new data."""
    lib.init_device(0, 48 * MB)
    bufs = _units(4, 8)
    s = lib.debug_stream_create(0)
    us = lib.UnitStream(0, [b.id for b in bufs], 16 * MB, True, 2)
    for _ in range(4):
        _pass(us, bufs, s)
    assert us.stats()["held"] >= 4
    lib.debug_stream_sync(s)
    bufs[1].write(torch.full((8 * MB,), 42, dtype=torch.uint8))
    bufs[1].set_preferred_location("cpu")  # a migration away from the held HBM copy
    bufs[1].prefetch("cpu")
    assert int(bufs[1].read()[0]) == 42
    lid, dptr = us.use(1, s)
    lib.debug_stream_sync(s)
    t = rt._tensor_from_ptr(dptr, (4096,), torch.uint8, "cpu", 0, bufs[1].id)
    assert int(t[0]) == 42 and int(t[-1]) == 42
    us.release(lid, s)
    lib.debug_stream_sync(s)
    del us
    lib.debug_stream_destroy(s)
    for b in bufs:
        b.free()


def test_shutdown_with_live_unit_stream(fake_rt):
    """A UnitStream still alive when the runtime shuts down (a model whose
    construction raised, a caller that never closed it) is detached by the
    shutdown: its holds go back first, and collecting it later touches nothing
    of the deleted runtime; its calls then fail cleanly."""
    lib.init_device(0, 48 * MB)
    bufs = _units(4, 8)
    s = lib.debug_stream_create(0)
    us = lib.UnitStream(0, [b.id for b in bufs], 16 * MB, True, 2)
    for _ in range(4):
        _pass(us, bufs, s)
    assert us.stats()["held"] >= 4
    lib.debug_stream_sync(s)
    lib.debug_stream_destroy(s)
    lib.shutdown()
    with pytest.raises(Exception):
        us.use(0, 0)
    del us  # must not crash (use-after-free of the runtime before the fix)
    rt.init("fake", fake_devices=2, fake_hbm_mb=64, lock_check=1, host_budget_mb=1024, pack_host_copies=0)
