"""Pluggable-allocator managed mode: torch allocations as evictable stable-VA
managed ranges (csrc/core/torch_allocator.cpp). On the fake backend the stable
VA is a CPU mapping of the fake HBM chunk, so contents are checked through it.
Parity target: cudaMallocManaged memory oversubscribing the GPU
(kernel-open/nvidia-uvm/uvm_migrate.c:882 prefetch, uvm_pmm_gpu.c eviction)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from ogkm import rt
from ogkm._native import RuntimeStatusError, lib

MB = 1 << 20


def _write(ptr: int, arr: np.ndarray) -> None:
    ctypes.memmove(ptr, arr.ctypes.data, arr.nbytes)


def _read(ptr: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int32)
    ctypes.memmove(out.ctypes.data, ptr, out.nbytes)
    return out


@pytest.fixture
def managed_rt(fake_rt):
    lib.configure("hbm_provider", 1)
    lib.configure("torch_alloc_managed_min_mb", 4)
    lib.init_device(0, 32 * MB)  # 16 chunks of fake HBM
    yield fake_rt


def test_managed_tensors_oversubscribe_and_keep_their_address(managed_rt):
    n = 8 * MB
    ptrs, refs = [], []
    for i in range(3):  # 3 x 8 MB active fits in 32 MB
        p = lib.torch_alloc(n, 0)
        ref = np.arange(n // 4, dtype=np.int32) * (i + 3)
        _write(p, ref)
        lib.torch_park(p, 0)
        ptrs.append(p)
        refs.append(ref)
    # 3 more tensors: 48 MB of tensors on a 32 MB arena - parked ones are evicted
    for i in range(3, 6):
        p = lib.torch_alloc(n, 0)
        ref = np.full(n // 4, i, dtype=np.int32)
        _write(p, ref)
        lib.torch_park(p, 0)
        ptrs.append(p)
        refs.append(ref)
    st = lib.torch_managed_stats(0)
    assert st["parked_bytes"] == 6 * n and st["active_bytes"] == 0
    assert lib.stats()["evictions"] > 0
    # every tensor comes back at its own address with its own contents
    for p, ref in zip(ptrs, refs):
        lib.torch_unpark(p, 0)
        assert np.array_equal(_read(p, n // 4), ref)
        lib.torch_park(p, 0)
    assert lib.torch_managed_stats(0)["unparks"] == 6
    # every remap of a stable VA ends with a GPU translation flush (tools/probe_vmm_tlb.hip:
    # unmap + map alone leaves stale translations on gfx950)
    st = lib.stats()
    assert st["vmm_remaps"] > 0 and st["tlb_flushes"] > 0 and st["vmm_errors"] == 0
    for p in ptrs:
        lib.torch_free(p, 0)
    rt.sync()
    lib.torch_alloc(1 * MB, 0)  # any allocation reaps deferred frees
    assert lib.torch_managed_stats(0)["parked_bytes"] == 0


def test_active_tensors_are_never_evicted(managed_rt):
    n = 8 * MB
    a = lib.torch_alloc(n, 0)
    _write(a, np.full(n // 4, 7, dtype=np.int32))
    parked = [lib.torch_alloc(n, 0) for _ in range(3)]
    for p in parked:
        lib.torch_park(p, 0)
    # a stays active while 3 more active tensors push every parked one out
    active = [lib.torch_alloc(n, 0) for _ in range(3)]
    assert all(active)
    assert np.array_equal(_read(a, n // 4), np.full(n // 4, 7, dtype=np.int32))
    assert lib.torch_managed_stats(0)["active_bytes"] == 4 * n
    # 32 MB of active tensors fill the arena: nothing evictable is left
    assert lib.torch_alloc(n, 0) == 0
    with pytest.raises(RuntimeStatusError):
        lib.torch_unpark(parked[0], 0)
    for p in [a] + parked + active:
        lib.torch_free(p, 0)


def test_small_allocations_stay_arena_extents(managed_rt):
    p = lib.torch_alloc(1 * MB, 0)
    assert lib.torch_managed_stats(0)["active_bytes"] == 0
    with pytest.raises(RuntimeStatusError):
        lib.torch_park(p, 0)  # not a managed allocation
    lib.torch_free(p, 0)


def test_partially_evicted_tensor_relocates_under_its_address(managed_rt):
    """Only part of a parked tensor is evicted; unpark relocates the resident
    part into a fresh extent (D2D) and faults the rest back: the stable VA must
    follow every block to its new chunk."""
    n = 8 * MB
    b = lib.torch_alloc(16 * MB, 0)     # chunks 0-7, active
    a = lib.torch_alloc(n, 0)           # chunks 8-11
    ref = np.arange(n // 4, dtype=np.int32) ^ 0x5A5A
    _write(a, ref)
    lib.torch_park(a, 0)
    c = lib.torch_alloc(12 * MB, 0)     # 6 contiguous chunks: 12-15 + two of a's
    assert c and lib.stats()["evictions"] >= 1
    info = lib.torch_managed_stats(0)
    assert info["parked_bytes"] == n
    lib.torch_free(b, 0)
    rt.sync()
    lib.torch_alloc(4096, 0)            # reaps b's deferred free
    lib.torch_unpark(a, 0)
    assert np.array_equal(_read(a, n // 4), ref)
    for p in (a, c):
        lib.torch_free(p, 0)


def test_op_holds_make_operands_resident_and_evictable_after(managed_rt):
    """The transparent mode's op protocol (torch_op_begin / torch_op_end): an
    op's managed operands are resident (and pinned) between begin and end, the
    outputs it allocated lose their allocation hold at end, and afterwards
    every tensor is evictable - 6 x 8 MB cycled through a 32 MB arena."""
    n = 8 * MB
    ptrs, refs = [], []
    for i in range(6):
        p = lib.torch_alloc(n, 0)
        ref = np.full(n // 4, 100 + i, dtype=np.int32)
        _write(p, ref)
        held, _ = lib.torch_op_begin([(p, True)], 0, 0)
        assert held == [p]
        lib.torch_op_end(held, [p], 0, 0)  # p is this op's output: its alloc hold goes too
        ptrs.append(p)
        refs.append(ref)
    st = lib.torch_managed_stats(0)
    assert st["active_bytes"] == 0 and st["parked_bytes"] == 6 * n
    for rnd in range(2):
        for i, p in enumerate(ptrs):
            q = ptrs[(i + 1) % 6]
            held, _ = lib.torch_op_begin([(p, False), (q, True), (12345, True)], 0, 0)  # non-managed ptr ignored
            assert sorted(held) == sorted([p, q])
            assert np.array_equal(_read(p, n // 4), refs[i])
            assert lib.torch_managed_stats(0)["active_bytes"] == 2 * n
            lib.torch_op_end(held, [], 0, 0)
    assert lib.stats()["evictions"] > 6
    for p in ptrs:
        lib.torch_free(p, 0)


def test_op_hold_nests_with_allocation_hold(managed_rt):
    n = 8 * MB
    p = lib.torch_alloc(n, 0)  # allocation hold
    held, pers = lib.torch_op_begin([(p, False), (p, True)], 0, 0)  # duplicate operand: one hold
    assert held == [p] and pers == []
    lib.torch_op_end(held, [], 0, 0)
    # its first use as an operand also ended its allocation hold
    assert lib.torch_managed_stats(0)["active_bytes"] == 0
    lib.configure("torch_persistent_ops", 3)
    tmp = [lib.torch_alloc(4 * MB, 0) for _ in range(3)]
    for t in tmp:  # three other ops later ...
        h, _ = lib.torch_op_begin([(t, False)], 0, 0)
        lib.torch_op_end(h, [], 0, 0)
    held, pers = lib.torch_op_begin([(p, False)], 0, 0)
    assert pers == [p]  # ... the second hold marks p long-lived (a parameter, not an activation)
    lib.torch_op_end(held, [], 0, 0)
    q = lib.torch_alloc(4 * MB, 0)
    tmp.append(q)
    held, pers = lib.torch_op_begin([(q, False)], 0, 0)
    lib.torch_op_end(held, [], 0, 0)
    held, pers = lib.torch_op_begin([(q, False)], 0, 0)
    assert pers == []  # held by consecutive ops: short-lived (an activation)
    lib.torch_op_end(held, [], 0, 0)
    for t in tmp:
        lib.torch_free(t, 0)
    assert lib.torch_managed_size(p, 0) == n and lib.torch_is_managed(p, 0)
    lib.torch_free(p, 0)


def test_recycled_activation_never_keys_the_trace(managed_rt):
    """A residual-stream activation lives ~35 ops and its address comes back
    every layer (the allocation cache): held at both ends of its life it must
    not count as long-lived (the stock 70B's 1 MB residual did, and the op
    trace saw its first repeat inside layer one); a parameter used once per
    pass does."""
    lib.configure("torch_persistent_ops", 64)
    try:
        w = lib.torch_alloc(8 * MB, 0)  # a parameter
        h, pers = lib.torch_op_begin([(w, False)], 0, 0)
        lib.torch_op_end(h, [], 0, 0)
        other = lib.torch_alloc(4 * MB, 0)
        addrs = set()
        for layer in range(6):
            x = lib.torch_alloc(4 * MB, 0)
            addrs.add(x)
            for j in range(40):
                ops = [(x, False)] if j in (0, 39) else [(other, False)]
                h, pers = lib.torch_op_begin(ops, 0, 0)
                assert x not in pers
                lib.torch_op_end(h, [], 0, 0)
            lib.torch_free(x, 0)
        assert len(addrs) < 6  # the address was recycled
        h, pers = lib.torch_op_begin([(w, False)], 0, 0)
        assert pers == [w]
        lib.torch_op_end(h, [], 0, 0)
        lib.torch_free(other, 0)
        lib.torch_free(w, 0)
    finally:
        lib.configure("torch_persistent_ops", 128)


@pytest.mark.parametrize("lazy", [0, 1])
def test_stable_placement_batches_evictions(managed_rt, lazy):
    """A stable-VA lease needs no contiguous extent: blocks take any chunk,
    victims go out as one batch per group, and a block that returns to its old
    chunk needs no remap (lazy unmap keeps the mapping)."""
    lib.configure("stable_lazy_unmap", lazy)
    lib.configure("stable_batch_blocks", 2)
    try:
        n = 12 * MB
        a = lib.torch_alloc(n, 0)
        _write(a, np.arange(n // 4, dtype=np.int32))
        lib.torch_park(a, 0)
        b = lib.torch_alloc(24 * MB, 0)  # 12 + 24 > 32: part of a is evicted
        lib.torch_park(b, 0)
        s0 = lib.stats()
        lib.torch_unpark(a, 0)
        assert np.array_equal(_read(a, n // 4), np.arange(n // 4, dtype=np.int32))
        s1 = lib.stats()
        assert s1["evictions"] > s0["evictions"]
        assert s1["vmm_errors"] == 0
        lib.torch_park(a, 0)
        for p in (a, b):
            lib.torch_free(p, 0)
    finally:
        lib.configure("stable_lazy_unmap", 0)
        lib.configure("stable_batch_blocks", 32)


def test_cyclic_remaps_elide_covered_flushes(managed_rt):
    """Cycling 6 x 8 MB tensors through a 32 MB arena: a block that comes back
    long after its eviction (a flush begun after its unmap has completed) is
    mapped without another translation flush; one that returns right away is
    flushed. Data stays right on every pass."""
    n = 8 * MB
    ptrs = []
    for i in range(6):
        p = lib.torch_alloc(n, 0)
        _write(p, np.full(n // 4, i, dtype=np.int32))
        lib.torch_park(p, 0)
        ptrs.append(p)
    s0 = lib.stats()
    for _ in range(4):
        for i, p in enumerate(ptrs):
            lib.torch_unpark(p, 0)
            assert int(_read(p, n // 4)[-1]) == i
            lib.torch_park(p, 0)
    s1 = lib.stats()
    remaps = s1["vmm_remaps"] - s0["vmm_remaps"]
    flushes = s1["tlb_flushes"] - s0["tlb_flushes"]
    elided = s1["tlb_flushes_elided"] - s0["tlb_flushes_elided"]
    assert remaps > 0 and elided > 0 and s1["vmm_errors"] == 0
    assert flushes < 24  # at most one per unpark; covered maps flush nothing
    for p in ptrs:
        lib.torch_free(p, 0)


def _cycle(ptrs, skip=()):
    """Hold each tensor for one read op (pushes the others out of a small arena)."""
    for p in ptrs:
        if p in skip:
            continue
        held, _ = lib.torch_op_begin([(p, False)], 0, 0)
        lib.torch_op_end(held, [], 0, 0)


def test_partial_write_dirties_only_written_pages(managed_rt):
    """A written view revokes the host copy of only the pages it writes: after
    a read brought the tensor back (duplicated), a one-row write followed by an
    eviction copies out those pages, not the tensor (per-page dirty state,
    uvm_va_block.h:101-230)."""
    lib.configure("perf_workingset_active_pct", 0)  # plain LRU: every tensor of the cycle is evicted each pass
    lib.init_device(0, 32 * MB)  # (the arena reads it at creation)
    n = 8 * MB
    p = lib.torch_alloc(n, 0)
    ref = np.arange(n // 4, dtype=np.int32)
    _write(p, ref)
    held, _ = lib.torch_op_begin([(p, True)], 0, 0)
    lib.torch_op_end(held, [p], 0, 0)
    others = [lib.torch_alloc(8 * MB, 0) for _ in range(4)]
    for q in others:
        held, _ = lib.torch_op_begin([(q, True)], 0, 0)
        lib.torch_op_end(held, [q], 0, 0)
    _cycle([p] + others)
    _cycle([p] + others)  # 5 x 8 MB cycled through 32 MB: every tensor was evicted, each has a host copy
    # read: resident in HBM as a duplicate of its host copy
    held, _ = lib.torch_op_begin([(p, False)], 0, 0)
    lib.torch_op_end(held, [], 0, 0)
    # write 3 scattered 1 KB rows (pages 1, 700, 1500) through a strided view
    rows = [1 * 4096 + 64, 700 * 4096 + 8, 1500 * 4096 + 1000]
    written = np.array([x for r in rows for x in (r & ~4095, (r & ~4095) + 4096)], dtype=np.int64)
    held, _ = lib.torch_op_begin([(p, True, rows[0], rows[-1] + 1024, written)], 0, 0)
    for r in rows:
        ref[r // 4:(r + 1024) // 4] = -7
        _write(p + r, np.full(256, -7, dtype=np.int32))
    lib.torch_op_end(held, [], 0, 0)
    assert lib.stats()["write_invalidations"] >= 2  # blocks 0 and 1 (page 1500 is in block 2... of 4)
    lib.sync_all()
    d0 = lib.stats()["bytes_xfer_dth"]
    _cycle(others)  # evicts p again
    lib.sync_all()
    dth = lib.stats()["bytes_xfer_dth"] - d0
    # the 3 written pages: the other tensors were only read since their last eviction (clean)
    assert dth == 3 * 4096, dth
    held, _ = lib.torch_op_begin([(p, False)], 0, 0)
    assert np.array_equal(_read(p, n // 4), ref)
    lib.torch_op_end(held, [], 0, 0)
    for q in others + [p]:
        lib.torch_free(q, 0)


def test_next_use_hints_evict_the_furthest_needed(managed_rt):
    """With next-use hints the arena evicts the tensor needed furthest in the
    future, whatever its recency (Belady order; LRU would pick `a`)."""
    ts = [lib.torch_alloc(8 * MB, 0) for _ in range(3)]
    a, b, c = ts
    for t in ts:  # written once, then each op ends; a is least recently used
        held, _ = lib.torch_op_begin([(t, True)], 0, 0)
        lib.torch_op_end(held, [t], 0, 0, [], 0)
    lib.torch_op_end([], [], 0, 0, [(a, 12), (b, 1000), (c, 11)], 10)
    d = lib.torch_alloc(16 * MB, 0)  # needs 2 of the 3: b (furthest) goes first, then ... not a/c both
    held, _ = lib.torch_op_begin([(d, True)], 0, 0)
    lib.torch_op_end(held, [d], 0, 0)
    info = {t: lib.torch_resident_bytes(t, 0) for t in ts}
    assert info[b] == 0, info
    assert info[a] + info[c] >= 8 * MB, info
    for t in ts + [d]:
        lib.torch_free(t, 0)


def test_prefetch_never_evicts_data_needed_sooner(managed_rt):
    ts = [lib.torch_alloc(8 * MB, 0) for _ in range(4)]  # 32 MB: the whole arena
    for t in ts:
        held, _ = lib.torch_op_begin([(t, True)], 0, 0)
        lib.torch_op_end(held, [t], 0, 0)
    lib.torch_op_end([], [], 0, 0, [(t, 20 + i) for i, t in enumerate(ts)], 10)
    e = lib.torch_alloc(8 * MB, 0)
    held, _ = lib.torch_op_begin([(e, True)], 0, 0)
    lib.torch_op_end(held, [e], 0, 0, [(e, 100)], 10)  # e needed last: it was written, one of ts went
    gone = [t for t in ts if lib.torch_resident_bytes(t, 0) < 8 * MB]
    assert gone == [ts[3]]  # the furthest-needed of ts (23) made room
    # prefetching ts[3] for time 23 may evict e (needed at 100) ...
    assert lib.torch_prefetch([(ts[3], 23)], 0) == 1
    lib.torch_prefetch_wait(0)
    lib.sync_all()
    assert lib.torch_resident_bytes(ts[3], 0) == 8 * MB and lib.torch_resident_bytes(e, 0) < 8 * MB
    # ... but prefetching e for time 100 must not evict anything needed before 100
    n0 = lib.stats()["evictions"]
    lib.torch_prefetch([(e, 100)], 0)
    lib.torch_prefetch_wait(0)
    lib.sync_all()
    assert all(lib.torch_resident_bytes(t, 0) == 8 * MB for t in ts)
    assert lib.stats()["evictions"] == n0
    for t in ts + [e]:
        lib.torch_free(t, 0)


def test_freed_tensor_eviction_copies_nothing(managed_rt):
    """A freed tensor's data is dead: evicting its chunks (in the reuse cache or
    awaiting its fence) copies nothing out, and a reuse does not copy it back."""
    lib.configure("torch_alloc_cache_mb", 64)
    p = lib.torch_alloc(8 * MB, 0)
    _write(p, np.ones(2 * MB, dtype=np.int32))
    held, _ = lib.torch_op_begin([(p, True)], 0, 0)
    lib.torch_op_end(held, [p], 0, 0)
    lib.torch_free(p, 0)
    lib.sync_all()
    s0 = lib.stats()
    big = [lib.torch_alloc(10 * MB, 0) for _ in range(3)]  # 30 MB: pushes the cached range out
    lib.sync_all()
    s1 = lib.stats()
    assert s1["evictions"] > s0["evictions"]
    assert s1["bytes_xfer_dth"] == s0["bytes_xfer_dth"]
    for q in big:
        lib.torch_free(q, 0)
    q = lib.torch_alloc(8 * MB, 0)  # a reuse of a cached range: nothing comes back over the link
    lib.sync_all()
    assert lib.stats()["bytes_xfer_htd"] == s1["bytes_xfer_htd"]
    lib.torch_free(q, 0)


def test_accessed_by_is_served_by_a_local_copy(managed_rt):
    """A remote (zero-copy) decision - accessed_by the GPU with the data resting
    in host DRAM - would not be mapped by the tensor's stable VA: the op hold
    falls back to a local copy instead of failing the op (uvm_va_block.c:11625-11664
    keeps such data remote; the stable VA maps HBM only)."""
    n = 8 * MB
    p = lib.torch_alloc(n, 0)
    ref = np.arange(n // 4, dtype=np.int32) * 3
    _write(p, ref)
    held, _ = lib.torch_op_begin([(p, True)], 0, 0)
    lib.torch_op_end(held, [p], 0, 0)
    lib.torch_set_read_mostly(p, 0, False)
    lib.torch_advise(p, 0, rt.ADVISE_SET_PREFERRED_LOCATION, 1, 0, 0)
    lib.torch_advise(p, 0, rt.ADVISE_SET_ACCESSED_BY, 0, 0, 0)
    others = [lib.torch_alloc(8 * MB, 0) for _ in range(4)]
    for q in others:
        held, _ = lib.torch_op_begin([(q, True)], 0, 0)
        lib.torch_op_end(held, [q], 0, 0)
    lib.sync_all()
    assert lib.torch_resident_bytes(p, 0) < n  # out in host DRAM
    f0 = lib.stats()["remote_fallbacks"]
    held, _ = lib.torch_op_begin([(p, False)], 0, 0)
    assert held == [p]
    assert np.array_equal(_read(p, n // 4), ref)
    lib.torch_op_end(held, [], 0, 0)
    assert lib.stats()["remote_fallbacks"] > f0
    for q in others + [p]:
        lib.torch_free(q, 0)


def test_stale_translations_are_flushed(managed_rt):
    """Fake translation model of gfx950 VMM (a remapped VA serves the old chunk
    until a flush): the init-time self-test sees the stale reads and that the
    flush cures them, and managed tensors cycled through the arena - every
    remap followed by the runtime's (elided where safe) flushes - keep their
    contents."""
    lib.inject("tlb_mode", 1)
    lib.init_device(0, 32 * MB)
    t = [a for a in lib.stats()["arenas"] if a["name"] == "hbm0"][0]["vmm_selftest"]
    assert t["ran"] and t["ok"] and t["flushed_ok"] == t["rounds"] > 0 and t["unflushed_stale"] > 0, t
    n = 8 * MB
    ptrs, refs = [], []
    for i in range(6):
        p = lib.torch_alloc(n, 0)
        assert lib.torch_is_managed(p, 0)
        ref = np.arange(n // 4, dtype=np.int32) * (i + 1)
        _write(p, ref)
        held, _ = lib.torch_op_begin([(p, True)], 0, 0)
        lib.torch_op_end(held, [p], 0, 0)
        ptrs.append(p)
        refs.append(ref)
    for rnd in range(3):
        for p, ref in zip(ptrs, refs):
            held, _ = lib.torch_op_begin([(p, False)], 0, 0)
            assert np.array_equal(_read(p, n // 4), ref)
            lib.torch_op_end(held, [], 0, 0)
    assert lib.stats()["vmm_remaps"] > 12 and lib.stats()["tlb_flushes"] > 0
    for p in ptrs:
        lib.torch_free(p, 0)
    lib.inject("tlb_mode", 0)


def test_failed_translation_self_test_refuses_managed_mode(managed_rt):
    """A GPU whose translation flush does not work fails the self-test: torch
    allocations stay plain arena extents (never read through a stale mapping)
    and ogkm.managed() refuses to start."""
    import ogkm

    lib.inject("tlb_mode", 2)
    try:
        lib.init_device(0, 32 * MB)
        t = [a for a in lib.stats()["arenas"] if a["name"] == "hbm0"][0]["vmm_selftest"]
        assert t["ran"] and not t["ok"] and "stale" in t["detail"], t
        p = lib.torch_alloc(8 * MB, 0)
        assert p and not lib.torch_is_managed(p, 0)
        lib.torch_free(p, 0)
        with pytest.raises(RuntimeError, match="self-test"):
            ogkm.managed(0)
    finally:
        lib.inject("tlb_mode", 0)
