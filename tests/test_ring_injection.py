"""SQ/CQ ring + failure injection (analog of uvm_channel_test.c RC recovery,
uvm_ce_test.c, and the UVM_TEST_*_INJECT_* error paths)."""
from __future__ import annotations

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20
CPU_TO_GPU, GPU_TO_CPU, GPU_INTERNAL, GPU_TO_GPU, MEMOPS, CXL = range(6)


def _dev_buf(nbytes, fill=None):
    b = rt.malloc_managed(nbytes, "devbuf")
    if fill is not None:
        b.fill(fill)
    l = b.acquire(0, rt.WRITE)
    l.wait(0)
    return b, l


def test_ring_copy_memset_and_cqes(fake_rt):
    a, la = _dev_buf(4 * MB, 0x01010101)
    b, lb = _dev_buf(4 * MB)
    seq = lib.ring_copy(0, GPU_INTERNAL, lb.dptr, la.dptr, 4 * MB, True)
    assert seq >= 1
    assert torch.equal(lb.tensor((4 * MB,), torch.uint8), la.tensor((4 * MB,), torch.uint8))
    lib.ring_memset(0, MEMOPS, lb.dptr, 0xDEADBEEF, 4 * MB)
    assert int(lb.tensor((MB,), torch.int32)[0]) == int(torch.tensor(0xDEADBEEF).to(torch.int32))
    cqes = lib.ring_reap(0, GPU_INTERNAL)
    assert cqes and all(st == 0 for _, _, st in cqes)
    ring = [r for r in lib.stats()["rings"] if r["dev"] == 0 and r["kind"] == "gpu_internal"][0]
    assert ring["completed"] >= ring["submitted"] >= seq
    la.release(0)
    lb.release(0)


def test_gather_scatter_pages(fake_rt):
    src = torch.arange(64 * 1024, dtype=torch.int32)
    dst = torch.zeros(8 * 1024, dtype=torch.int32)
    pages = [1, 3, 5, 8, 13, 21, 34, 55]
    lib.ring_gather(0, src.data_ptr(), dst.data_ptr(), pages, 4096, False)
    assert torch.equal(dst, torch.cat([src[p * 1024:(p + 1) * 1024] for p in pages]))
    back = torch.zeros_like(src)
    lib.ring_gather(0, back.data_ptr(), dst.data_ptr(), pages, 4096, True)
    for p in pages:
        assert torch.equal(back[p * 1024:(p + 1) * 1024], src[p * 1024:(p + 1) * 1024])


def test_copy_drop_injection_reports_error(fake_rt):
    """A dropped copy (simulated link error) surfaces as an error CQE and a sticky
    ring error with the push description, not as silent corruption."""
    b = rt.malloc_managed(2 * MB, "drop")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    lib.inject("copy_drop", 1)
    with pytest.raises(rt.RuntimeStatusError, match="INJECTED_ERROR"):
        b.migrate("gpu:0")
    st, desc = lib.ring_error(0, CPU_TO_GPU)
    assert st == "INJECTED_ERROR" and "migrate.cpp" in desc
    assert lib.stats()["injected_errors"] == 1
    lib.ring_clear_error(0, CPU_TO_GPU)
    b.migrate("gpu:0")  # recovered
    assert int(b.read().min()) == 1


def test_copy_drop_behind_queued_batch_never_hangs_waiters(fake_rt):
    """A copy dropped while an earlier SDMA batch is still queued: the ring's
    tracking value stays monotonic (the error batch is published in order after
    the slow one), so waits on every sequence number return - the error, not a
    hang (the direct store raced the worker's smaller stores)."""
    import time

    src = torch.ones(4 * MB, dtype=torch.uint8)
    dst = torch.zeros(4 * MB, dtype=torch.uint8)
    rt.configure(fake_dma_delay_us=200_000)
    try:
        s1 = lib.ring_copy(0, CPU_TO_GPU, dst.data_ptr(), src.data_ptr(), 2 * MB, False)
        lib.inject("copy_drop", 1)
        s2 = lib.ring_copy(0, CPU_TO_GPU, dst.data_ptr() + 2 * MB, src.data_ptr() + 2 * MB, 2 * MB, False)
        assert s2 > s1
        t0 = time.time()
        assert lib.ring_wait_seq(0, CPU_TO_GPU, s2) == "INJECTED_ERROR"
        assert lib.ring_wait_seq(0, CPU_TO_GPU, s1) == "INJECTED_ERROR"
        assert time.time() - t0 < 5
        # The value never moves backwards once published.
        c = lib.ring_completed(0, CPU_TO_GPU)
        assert c >= s2
        time.sleep(0.3)
        assert lib.ring_completed(0, CPU_TO_GPU) >= c
    finally:
        rt.configure(fake_dma_delay_us=0)
        lib.ring_clear_error(0, CPU_TO_GPU)


def test_failure_after_submission_is_caught_at_completion(fake_rt):
    """A copy that fails after it was submitted (ECC / link error, faulting
    kernel) is caught when its completion is checked: the fence wait returns the
    error, the CQE retired with it carries the status, the ring records it
    (uvm_channel.c:2047-2112 channel error detection)."""
    from ogkm import tools

    q = tools.EventQueue(events=["RingError"])
    b = rt.malloc_managed(2 * MB, "late")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    lib.ring_reap(0, CPU_TO_GPU)
    lib.inject("async_copy_error", 1)
    with pytest.raises(rt.RuntimeStatusError, match="INJECTED_ERROR"):
        b.migrate("gpu:0")
    cqes = lib.ring_reap(0, CPU_TO_GPU)
    assert any(st != 0 for _, _, st in cqes)
    assert lib.ring_error(0, CPU_TO_GPU)[0] == "INJECTED_ERROR"
    assert any(e["type"] == "RingError" for e in q.read_dicts())
    q.close()
    lib.ring_clear_error(0, CPU_TO_GPU)
    b.migrate("gpu:0")
    assert int(b.read().min()) == 1


def test_alloc_fail_after_and_recovery(fake_rt):
    lib.init_device(0, 32 * MB)
    lib.inject("alloc_fail_after", 0)
    b = rt.malloc_managed(4 * MB, "af")
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    with pytest.raises(rt.RuntimeStatusError):
        b.migrate("gpu:0")
    lib.inject("alloc_fail_after", -1)
    b.migrate("gpu:0")
    assert lib.arena_check(0, 0) == ""


def test_evict_fail_injection(fake_rt):
    lib.init_device(0, 8 * MB)
    a = rt.malloc_managed(8 * MB, "a")
    a.fill(7)
    a.migrate("gpu:0")
    lib.inject("evict_fail", 1)
    b = rt.malloc_managed(8 * MB, "b")
    b.fill(9)
    with pytest.raises(rt.RuntimeStatusError):
        b.migrate("gpu:0")
    b.migrate("gpu:0")  # the next attempt evicts normally
    assert int(a.read()[0]) == 7
    assert lib.arena_check(0, 0) == ""


def test_populate_and_host_alloc_errors(fake_rt):
    b = rt.malloc_managed(2 * MB, "pe")
    lib.inject("host_alloc_error", 1)
    with pytest.raises(rt.RuntimeStatusError):
        b.write(torch.ones(2 * MB, dtype=torch.uint8))
    lib.inject("populate_error", 1)
    with pytest.raises(rt.RuntimeStatusError):
        b.write(torch.ones(2 * MB, dtype=torch.uint8))
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    assert int(b.read().sum()) == 2 * MB


def test_ring_backpressure_small_queue(fake_rt):
    """More SQEs than entries: push() submits and waits instead of overflowing."""
    lib.shutdown()
    lib.config_reset()
    rt.init("fake", fake_devices=1, fake_hbm_mb=64, lock_check=1, channel_num_gpfifo_entries=8)
    src = torch.arange(1 << 20, dtype=torch.uint8)
    dst = torch.zeros_like(src)
    for i in range(64):
        lib.ring_copy(0, GPU_INTERNAL, dst.data_ptr() + i * 16384, src.data_ptr() + i * 16384, 16384, False)
    lib.sync_all()
    assert torch.equal(dst, src)


def test_quiesce_blocks_new_faults(fake_rt):
    b = rt.malloc_managed(2 * MB, "q")
    b.fill(1)
    lib.quiesce()
    with pytest.raises(rt.RuntimeStatusError, match="BUSY"):
        b.acquire(0, rt.READ)
    lib.resume()
    b.acquire(0, rt.READ).release(0)


def test_lock_checker_detects_inversion(fake_rt):
    assert lib.lock_check_self_test() == 1
    lib.reset_lock_violations()  # the fixture asserts zero afterwards


def test_ecc_uncorrectable_error_is_fatal(fake_rt):
    """RAS counters are baselined at init; correctable errors are reported only,
    a new uncorrectable (ECC or xGMI link) error makes the runtime FATAL - the
    reference's ECC notifier check after pushes (uvm_gpu.c:1328-1354)."""
    h = lib.device_health(0)
    assert h["reported"] and h["status"] == "OK" and h["now"]["source"] == "fake"
    lib.inject_ras(0, 5, 0)            # correctable: counted, not fatal
    h = lib.device_health(0)
    assert h["now"]["ce"] == 5 and h["status"] == "OK"
    lib.inject_ras(0, 5, 1)            # one uncorrectable xGMI link error
    assert lib.device_health(0)["status"] == "FATAL"
    assert "xGMI" in lib.fatal_reason()
    with pytest.raises(Exception):
        rt.malloc_managed(1 << 20, "after-ecc")  # every later operation fails fast


def test_merged_batches_copy_after_staged_decode_into_same_chunk(fake_rt):
    """Two submissions the H2D worker merges into one batch: the first decodes
    a packed block into chunk E (staged: SDMA into HBM staging, decode after
    the copies landed), the second - after E was handed to another block -
    copies raw data into E. copy_pages skips same-ring fences (the ring is in
    order), so the batch itself must land the older decode first; before the
    fix the raw copy went out with the staging copies and the decode launched
    after them overwrote it (the transparent-mode packed training test's
    corrupted gradient)."""
    lib.configure("ans_stage_mb", 8)
    lib.configure("ring_merge_packed_mb", 64)  # (off by default)
    vals = lambda seed: (torch.randn(MB, generator=torch.Generator().manual_seed(seed)) * 0.02).to(torch.bfloat16)
    w1, w2, g = vals(1), vals(2), vals(3)
    enc1 = torch.frombuffer(bytearray(lib.ans_encode(w1.view(torch.uint8).numpy().tobytes())), dtype=torch.uint8)
    enc2 = torch.frombuffer(bytearray(lib.ans_encode(w2.view(torch.uint8).numpy().tobytes())), dtype=torch.uint8)
    assert 0 < enc1.numel() < 2 * MB and 0 < enc2.numel() < 2 * MB
    e, le = _dev_buf(2 * MB, 0)
    f, lf = _dev_buf(2 * MB, 0)
    # the worker is held in a first submission waiting on a slow stream
    s = lib.debug_stream_create(0)
    blk, lblk = _dev_buf(2 * MB, 0)
    lib.debug_touch(s, lblk.dptr, 2 * MB, 300000)
    lib.debug_ring_submit(0, CPU_TO_GPU, [(2, 0, s, 0, 0)])
    lib.debug_ring_submit(0, CPU_TO_GPU, [(1, le.dptr, enc1.data_ptr(), enc1.numel(), MB)])
    last = lib.debug_ring_submit(0, CPU_TO_GPU, [(1, lf.dptr, enc2.data_ptr(), enc2.numel(), MB),
                                                (0, le.dptr, g.data_ptr(), 2 * MB, 0)])
    assert lib.ring_wait_seq(0, CPU_TO_GPU, last) == "OK"
    assert lib.stats()["ring_merged_batches"] >= 1  # (the case under test)
    assert torch.equal(lf.tensor((MB,), torch.bfloat16).cpu(), w2)
    assert torch.equal(le.tensor((MB,), torch.bfloat16).cpu(), g)
    lib.debug_stream_sync(s)
    lib.debug_stream_destroy(s)
    for l in (le, lf, lblk):
        l.release(0)
