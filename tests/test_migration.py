"""Migration engine tests (fake backend): residency state machine, read
duplication, CPU faults through the CPU view, eviction write-back, 3-tier
demotion, prefetch / two-pass migrate, and the software fault batch service.
Modelled on the reference's UVM_TEST_VA_RESIDENCY_INFO-driven tests."""
from __future__ import annotations

import time

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20


def tiers(b, off=0):
    return sorted((r["tier"], r["id"]) for r in b.residency(off)["resident_on"])


def test_write_read_roundtrip_partial_pages(fake_rt):
    b = rt.malloc_managed(3 * MB + 123, "w")
    data = torch.randint(0, 256, (b.size,), dtype=torch.uint8)
    b.write(data[:1000], 0)
    b.write(data[1000:], 1000)  # unaligned split
    assert torch.equal(b.read(), data)
    # unpopulated buffers read as zeros
    z = rt.malloc_managed(5000, "z")
    assert int(z.read().sum()) == 0
    b.free()
    z.free()


def test_migrate_two_pass_and_back(fake_rt):
    b = rt.malloc_managed(6 * MB, "m")
    ref = torch.arange(6 * MB // 4, dtype=torch.int32)
    b.write(ref)
    assert tiers(b) == [("host", 0)]
    b.migrate("gpu:1")
    assert tiers(b) == [("gpu", 1)]
    b.migrate("host:0")
    assert tiers(b) == [("host", 0)]
    assert torch.equal(b.read().view(torch.int32), ref)
    s = lib.stats()
    assert s["bytes_xfer_htd"] >= 6 * MB and s["bytes_xfer_dth"] >= 6 * MB
    b.free()


def test_read_duplication_and_write_collapse(fake_rt):
    b = rt.malloc_managed(4 * MB, "rd")
    b.write(torch.full((4 * MB,), 5, dtype=torch.uint8))
    b.set_read_mostly(True)
    l = b.acquire(0, rt.READ)
    l.wait(0)
    l.release(0)
    info = b.residency(0)
    assert info["read_dup"] and ("gpu", 0) in tiers(b) and ("host", 0) in tiers(b)
    # A CPU write through the CPU view collapses duplication (revocation).
    v = b.cpu_view()
    v[0] = 9
    assert int(v[0]) == 9
    assert lib.stats()["revocations"] >= 1
    # the GPU copy of page 0 is gone; reacquire brings the new value
    l = b.acquire(0, rt.READ, 0, 4096)
    l.wait(0)
    assert int(l.tensor((4096,), torch.uint8)[0]) == 9
    l.release(0)
    b.free()


def test_cpu_fault_migrates_gpu_data_back(fake_rt):
    b = rt.malloc_managed(5 * MB, "cf")
    l = b.acquire(0, rt.WRITE)
    l.wait(0)
    l.tensor((5 * MB // 4,), torch.int32).copy_(torch.arange(5 * MB // 4, dtype=torch.int32))
    l.release(0)
    assert tiers(b) == [("gpu", 0)]
    v = b.cpu_view(torch.int32)
    assert int(v[12345]) == 12345  # SIGSEGV -> cpu_fault -> migrate -> map
    assert lib.stats()["cpu_page_faults"] >= 1
    assert ("host", 0) in tiers(b)
    assert torch.equal(v.clone(), torch.arange(5 * MB // 4, dtype=torch.int32))
    b.free()


def test_eviction_writes_back_dirty_data(fake_rt):
    lib.init_device(0, 8 * MB)  # 4 chunks
    a = rt.malloc_managed(6 * MB, "a")
    la = a.acquire(0, rt.WRITE)
    la.wait(0)
    la.tensor((6 * MB,), torch.uint8).fill_(7)
    la.release(0)
    b = rt.malloc_managed(6 * MB, "b")
    lb = b.acquire(0, rt.WRITE)  # forces eviction of `a` (its only copy is on the GPU)
    lb.wait(0)
    lb.release(0)
    assert ("gpu", 0) not in tiers(a)
    assert lib.stats()["bytes_xfer_dth"] >= 4 * MB
    assert int(a.read().min()) == 7
    a.free()
    b.free()


def test_three_tier_demotion_to_cxl(fake_rt):
    lib.cxl_rediscover(0, "/sys")  # emulate NUMA node 0 as a CXL pool
    lib.configure("host_budget_mb", 8)  # tiny host tier: 4 chunks
    lib.init_device(0, 8 * MB)
    bufs = []
    for i in range(6):  # 12 chunks of data: 4 fit in HBM, 4 in host, the rest must go to CXL
        b = rt.malloc_managed(4 * MB, f"t{i}")
        l = b.acquire(0, rt.WRITE)
        l.wait(0)
        l.tensor((4 * MB,), torch.uint8).fill_(i + 1)
        l.release(0)
        bufs.append(b)
    placed = [tiers(b) for b in bufs]
    assert any(("cxl", 0) in p for p in placed), placed
    for i, b in enumerate(bufs):
        assert int(b.read().max()) == i + 1
        b.free()


def test_preferred_location_cxl(fake_rt):
    lib.cxl_rediscover(0, "/sys")
    b = rt.malloc_managed(2 * MB, "c")
    b.set_preferred_location("cxl:0")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    assert tiers(b) == [("cxl", 0)]
    assert rt.mem_range_get_attribute(b, "preferred_location") == rt.Loc("cxl", 0)
    b.free()


def test_preferred_host_is_mapped_remotely(fake_rt):
    """UVM rule: a GPU fault on data preferring host keeps it there and maps it remotely."""
    b = rt.malloc_managed(4 * MB, "remote")
    b.set_preferred_location("host:0")
    b.set_accessed_by(0)
    b.write(torch.full((4 * MB,), 3, dtype=torch.uint8))
    l = b.acquire(0, rt.READ)
    assert l.remote
    l.wait(0)
    assert int(l.tensor((4 * MB,), torch.uint8)[-1]) == 3
    l.release(0)
    assert tiers(b) == [("host", 0)]
    assert lib.stats()["map_remote"] >= 1
    b.free()


def test_prefetch_async_tracker(fake_rt):
    b = rt.malloc_managed(8 * MB, "p")
    b.write(torch.ones(8 * MB, dtype=torch.uint8))
    tr = rt.mem_prefetch_async(b, "gpu:0")
    tr.wait()
    assert tr.query()
    assert tiers(b) == [("gpu", 0)]
    assert lib.stats()["prefetch_bytes_htd"] == 8 * MB
    b.free()


def test_fault_batch_coalescing_and_prefetch(fake_rt):
    b = rt.malloc_managed(2 * MB, "fb")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    faults = [(b.id, 0, 4096, 0, rt.READ)] * 5 + [(b.id, 4096 * p, 4096, 0, rt.READ) for p in range(1, 300)]
    lib.service_faults(faults)
    s = lib.stats()
    assert s["faults_coalesced"] == 4
    assert s["fault_batches"] == 1
    # 300 of 512 pages faulted (>51%): the prefetcher pulls the whole block
    assert b.residency(0)["resident_on"][-1]["pages"] == 512


def test_prefetch_hint_bitmap_tree(fake_rt):
    # 1 faulted page alone: nothing beyond it.
    assert lib.prefetch_hint([], [10], 512, 51) == [10]
    # 2 of 2 in an aligned pair -> the pair; then larger regions need >51%.
    h = lib.prefetch_hint(list(range(0, 200)), [200], 512, 51)
    assert h == list(range(0, 256))  # 201/256 > 51% of the 256-page subregion
    h = lib.prefetch_hint(list(range(0, 300)), [300], 512, 51)
    assert h == list(range(512))


def test_thrashing_detection_pins_block(fake_rt):
    lib.configure("perf_thrashing_threshold", 3)
    lib.configure("perf_thrashing_pin_threshold", 2)
    lib.configure("perf_thrashing_lapse_usec", 50_000)
    b = rt.malloc_managed(2 * MB, "th")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    for i in range(8):
        lib.service_faults([(b.id, 0, 4096, i % 2, rt.WRITE)])  # ping-pong GPU0 <-> GPU1
    s = lib.stats()
    assert s["thrashing_detected"] >= 1
    assert s["pin_events"] >= 1
    assert b.residency(0)["pinned"]
    b.free()


def test_range_group_freezes_residency(fake_rt):
    g = rt.create_range_group(migratable=False)
    b = rt.malloc_managed(2 * MB, "rg")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    b.set_range_group(g)
    with pytest.raises(rt.RuntimeStatusError):
        b.prefetch("gpu:0")
    rt.set_range_group_migratable(g, True)
    b.prefetch("gpu:0").wait()
    assert ("gpu", 0) in tiers(b)
    b.free()


def test_peer_migration_staged_when_link_down(fake_rt):
    b = rt.malloc_managed(4 * MB, "peer")
    b.write(torch.full((4 * MB,), 4, dtype=torch.uint8))
    b.migrate("gpu:0")
    lib.inject("peer_link_down", 1)  # GPU0's peer link is down: stage through host
    b.migrate("gpu:1")
    assert ("gpu", 1) in tiers(b)
    assert int(b.read().min()) == 4
    assert lib.stats()["bytes_xfer_dth"] >= 4 * MB  # the bounce through host memory
    b.free()


def test_stable_va_fake_vmm(fake_rt):
    lib.configure("hbm_provider", 1)
    lib.init_device(0, 16 * MB)
    b = rt.malloc_managed(4 * MB, "st", stable_va=True, device=0)
    b.write(torch.arange(1 << 20, dtype=torch.int32))
    b.migrate("gpu:0")
    t = rt._tensor_from_ptr(b.dev_va, (1 << 20,), torch.int32, "cpu")  # stable VA aliases the HBM chunk
    assert torch.equal(t, torch.arange(1 << 20, dtype=torch.int32))
    del t
    b.free()


def test_external_and_device_p2p_ranges(fake_rt):
    e = rt.alloc_device_p2p(4 * MB, 1, "p2p")
    info = lib.range_info(e.id)
    assert info["type"] == "device_p2p" and info["ext_ptr"]
    l = e.acquire(0, rt.READ)
    assert l.remote and l.dptr == info["ext_ptr"]
    l.release(0)
    x = rt.map_external(info["ext_ptr"], 4 * MB, 1, "ext")
    assert lib.range_info(x.id)["type"] == "external"
    assert x.residency(0)["resident_on"][0] == {"tier": "gpu", "id": 1, "pages": 512, "chunk": -1}
    x.free()
    e.free()


def test_ring_gather_scatter_memset_cpu(fake_rt):
    """Page-list pack/unpack and memset SQEs through a ring (fake backend)."""
    import torch

    src = torch.arange(64 * 1024, dtype=torch.int32)
    dst = torch.zeros(16 * 1024, dtype=torch.int32)
    idx = [3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59]
    lib.ring_gather(0, src.data_ptr(), dst.data_ptr(), idx, 4096, False)
    assert torch.equal(dst, torch.cat([src[i * 1024:(i + 1) * 1024] for i in idx]))
    back = torch.zeros_like(src)
    lib.ring_gather(0, back.data_ptr(), dst.data_ptr(), idx, 4096, True)
    for i in idx:
        assert torch.equal(back[i * 1024:(i + 1) * 1024], src[i * 1024:(i + 1) * 1024])
    m = torch.empty(1 << 16, dtype=torch.int32)
    lib.ring_memset(0, 4, m.data_ptr(), 0x7F7F7F7F, m.numel() * 4)
    assert bool((m == 0x7F7F7F7F).all())


def test_thrashing_throttle_then_pin_via_perf_bus(fake_rt):
    """GPU0 <-> CPU write ping-pong on one block: the thrashing module (a perf
    bus subscriber) detects it, throttles the processor that keeps pulling the
    block - its next fault maps the host copy remotely instead of migrating -
    ends the throttle after the nap, and finally pins the block
    (uvm_perf_thrashing.c:1535-1762, consumed as at uvm_va_block.c:12528)."""
    from ogkm import tools

    lib.configure("perf_thrashing_threshold", 3)
    lib.configure("perf_thrashing_pin_threshold", 4)
    lib.configure("perf_thrashing_lapse_usec", 50_000)   # nap = 1 lapse = 50 ms
    q = tools.EventQueue(events=["ThrashingDetected", "ThrottlingStart", "ThrottlingEnd", "MapRemote"])
    b = rt.malloc_managed(2 * MB, "pp")
    b.write(torch.ones(2 * MB, dtype=torch.uint8))
    procs = [0, rt.CPU, 0, rt.CPU, 0]          # the 4th migration throttles the CPU, the 5th the GPU
    for p in procs:
        lib.service_faults([(b.id, 0, 4096, p, rt.WRITE)])
    assert lib.stats()["thrashing_detected"] >= 1
    # the GPU is napping: its fault on a page still on the host maps it remotely
    mr0 = lib.stats()["map_remote"]
    lib.service_faults([(b.id, 8 * 4096, 4096, 0, rt.READ)])
    assert lib.stats()["map_remote"] == mr0 + 1
    assert not any(r["tier"] == "gpu" and r["pages"] > 1 for r in b.residency(0)["resident_on"])
    time.sleep(0.06)                           # the nap ends
    for p in [rt.CPU, 0, rt.CPU, 0, rt.CPU, 0]:
        lib.service_faults([(b.id, 0, 4096, p, rt.WRITE)])
    ev = [e["type"] for e in q.read_dicts()]
    q.close()
    assert "ThrashingDetected" in ev and "ThrottlingStart" in ev and "MapRemote" in ev and "ThrottlingEnd" in ev
    assert ev.index("ThrottlingStart") < ev.index("MapRemote") < ev.index("ThrottlingEnd")
    assert lib.stats()["pin_events"] >= 1 and b.residency(0)["pinned"]
    b.free()


def test_fragmented_block_copy_is_one_page_list_kernel(fake_rt):
    """A block whose faulted pages form many runs moves with one page-list
    copy (the LDS-staged k_page_copy_lds on a GPU) instead of one copy per run,
    and the data is exact."""
    lib.configure("perf_prefetch_enable", 0)
    b = rt.malloc_managed(2 * MB, "frag")
    ref = torch.randint(0, 256, (2 * MB,), dtype=torch.uint8)
    b.write(ref)
    pages = list(range(0, 512, 3))            # 171 single-page runs
    lib.service_faults([(b.id, p * 4096, 4096, 0, rt.READ) for p in pages])
    s = lib.stats()
    assert s["page_list_copies"] == 1
    gpu = [r for r in b.residency(0)["resident_on"] if r["tier"] == "gpu"]
    assert gpu and gpu[0]["pages"] == len(pages)
    l = b.acquire(0, rt.READ)                  # the rest comes in; every byte matches
    l.wait()
    assert torch.equal(l.tensor((2 * MB,), torch.uint8).clone(), ref)
    l.release()
    b.free()


def test_busy_cpu_fault_retried_later_without_blocking_others(fake_rt):
    """A CPU fault on a block whose only copy a GPU lease pins is BUSY: the
    service thread retries it in a LATER batch (uvm_va_space.c:2540-2590
    retries) while other posted faults complete right away; it completes once
    the lease is released."""
    import ctypes
    import threading
    import time

    a = rt.malloc_managed(2 * MB, "busy")
    la = a.acquire(0, rt.WRITE)
    la.wait(0)
    la.tensor((2 * MB // 4,), torch.int32).fill_(11)
    b = rt.malloc_managed(2 * MB, "free")
    b.write(torch.full((2 * MB // 4,), 22, dtype=torch.int32))
    lb = b.acquire(0, rt.READ)                     # GPU copy only while leased ...
    lb.wait(0)
    lb.release(0)
    va, vb = a.cpu_view(torch.int32), b.cpu_view(torch.int32)
    got = {}

    def touch(name, view):
        buf = ctypes.c_int32()
        ctypes.memmove(ctypes.addressof(buf), view.data_ptr() + 4096, 4)   # faults with the GIL released
        got[name] = (buf.value, time.perf_counter())

    t0 = time.perf_counter()
    ta = threading.Thread(target=touch, args=("a", va))
    ta.start()
    time.sleep(0.05)                                # a's fault is posted and BUSY
    tb = threading.Thread(target=touch, args=("b", vb))
    tb.start()
    tb.join(5)
    assert "b" in got and got["b"][0] == 22 and "a" not in got
    time.sleep(0.05)
    la.release(0)                                   # now a's retry succeeds
    ta.join(10)
    assert got["a"][0] == 11 and got["a"][1] > got["b"][1]
    assert time.perf_counter() - t0 < 10
    a.free()
    b.free()


@pytest.mark.parametrize("clean_first", [1, 0])
def test_eviction_prefers_clean_copies(fake_rt, clean_first):
    """HBM LRU with evict_clean_first: among GPU-preferred data (the managed
    torch tensors' advice), a block that still has a valid host copy
    (read-mostly data) is evicted before an older block whose only copy is in
    HBM (written there) - the clean victim costs no copy-out."""
    lib.configure("evict_clean_first", clean_first)
    lib.init_device(0, 16 * MB)  # 8 chunks
    dirty = rt.malloc_managed(8 * MB, "dirty")
    dirty.set_preferred_location("gpu:0")
    dirty.write(torch.full((2 * MB,), 3, dtype=torch.int32))
    l = dirty.acquire(0, rt.WRITE)  # written on the GPU: the host copy is gone
    l.release(0)
    clean = rt.malloc_managed(8 * MB, "clean")
    clean.write(torch.full((2 * MB,), 5, dtype=torch.int32))  # on the host
    clean.set_preferred_location("gpu:0")
    clean.set_read_mostly(True)
    l = clean.acquire(0, rt.READ)  # read-duplicated: host copy stays valid
    l.release(0)
    rt.sync()
    d0 = lib.stats()["bytes_xfer_dth"]
    third = rt.malloc_managed(8 * MB, "third")
    third.write(torch.full((2 * MB,), 7, dtype=torch.int32))
    l = third.acquire(0, rt.READ)  # needs 4 chunks: evicts 4 of the 8
    l.release(0)
    rt.sync()
    dth = lib.stats()["bytes_xfer_dth"] - d0
    if clean_first:
        assert dth == 0  # the newer but clean blocks went first
    else:
        assert dth >= 8 * MB  # plain LRU: the older dirty blocks were copied out
    assert int(dirty.read().view(torch.int32).min()) == 3 and int(clean.read().view(torch.int32).min()) == 5
    for b in (dirty, clean, third):
        b.free()
