"""GPU tests of the runtime on a real MI355X (HIP backend).

Numerics of every copy path are checked bit-exactly against a plain PyTorch
reference of the same data (copies must be exact). Modelled on the reference's
CE tests (uvm_ce_test.c:44-1258: memcpy/memset across apertures and sizes, CPU<->GPU
round trips) and PMM eviction tests (uvm_pmm_test.c).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

pytestmark = pytest.mark.gpu

MB = 1 << 20


def _rand_bytes(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g)


def test_backend_is_hip(gpu_rt):
    assert lib.backend_name() == "hip"
    assert lib.device_count() >= 1


@pytest.mark.parametrize("nbytes", [4096, 3 * MB + 4096, 37 * MB])
def test_host_to_gpu_roundtrip_exact(gpu_rt, nbytes):
    ref = _rand_bytes(nbytes, seed=nbytes)
    b = rt.malloc_managed(nbytes, "rt")
    b.write(ref)
    assert b.residency(0)["resident_on"][0]["tier"] == "host"
    with b.acquire(0, rt.READ) as l:
        t = l.tensor((nbytes,), torch.uint8)
        torch.cuda.synchronize()
        assert torch.equal(t.cpu(), ref)
    assert lib.stats()["bytes_xfer_htd"] >= nbytes
    b.free()


def test_gpu_write_then_cpu_fault(gpu_rt):
    n = 8 * MB
    b = rt.malloc_managed(n, "w")
    with b.acquire(0, rt.WRITE) as l:
        t = l.tensor((n // 4,), torch.float32)
        t.copy_(torch.arange(n // 4, dtype=torch.float32, device="cuda"))
        torch.cuda.synchronize()
    v = b.cpu_view(torch.float32)
    # Touching the CPU view faults the data back to host memory (SIGSEGV path).
    assert torch.equal(v[:1000].clone(), torch.arange(1000, dtype=torch.float32))
    assert float(v[-1]) == float(n // 4 - 1)
    assert lib.stats()["cpu_page_faults"] > 0
    b.free()


def test_eviction_under_budget(gpu_rt):
    lib.init_device(0, 64 * MB)
    bufs, refs = [], []
    for i in range(4):
        ref = _rand_bytes(40 * MB, seed=i)
        b = rt.malloc_managed(40 * MB, f"e{i}")
        b.write(ref)
        bufs.append(b)
        refs.append(ref)
    for rnd in range(2):
        for b, ref in zip(bufs, refs):
            with b.acquire(0, rt.WRITE) as l:
                t = l.tensor((40 * MB,), torch.uint8)
                torch.cuda.synchronize()
                assert torch.equal(t.cpu(), ref)
    s = lib.stats()
    assert s["evictions"] > 0
    assert lib.arena_check(0, 0) == ""
    for b in bufs:
        b.free()


def test_read_mostly_streaming_is_clean(gpu_rt):
    """Read-duplicated data is dropped (not copied back) when evicted."""
    lib.init_device(0, 32 * MB)
    b = rt.malloc_managed(96 * MB, "rm")
    ref = _rand_bytes(96 * MB, seed=7)
    b.write(ref)
    b.set_read_mostly(True)
    dth0 = lib.stats()["bytes_xfer_dth"]
    for off in range(0, 96 * MB, 16 * MB):
        l = b.acquire(0, rt.READ, off, 16 * MB)
        l.wait()
        t = l.tensor((16 * MB,), torch.uint8)
        torch.cuda.synchronize()
        assert torch.equal(t.cpu(), ref[off:off + 16 * MB])
        l.release()
    assert lib.stats()["bytes_xfer_dth"] == dth0
    b.free()


def test_ring_copy_bandwidth_h2d(gpu_rt):
    """The HIP copy kernel must saturate PCIe Gen5 H2D from the pinned host tier."""
    n = 1 << 30
    b = rt.malloc_managed(n, "bw")
    b.fill(0x01020304)
    b.set_read_mostly(True)
    lib.init_device(0, 2 << 30)
    l = b.acquire(0, rt.READ)
    l.wait()
    torch.cuda.synchronize()
    l.release()
    b.evict("gpu:0")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    l = b.acquire(0, rt.READ)
    l.wait(0)
    dt = time.perf_counter() - t0
    l.release()
    gbps = n / dt / 1e9
    print(f"acquire 1 GiB H2D: {gbps:.1f} GB/s")
    assert gbps > 50  # SDMA engine: ~56.8 GB/s on the box (profiles/r2_probe_sdma.txt)
    b.free()


def test_memset_and_gather_kernels(gpu_rt):
    src = torch.arange(64 * 1024, dtype=torch.int32, device="cuda")  # 64 pages of 4 KB
    dst = torch.zeros(16 * 1024, dtype=torch.int32, device="cuda")
    idx = [3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59]
    lib.ring_gather(0, src.data_ptr(), dst.data_ptr(), idx, 4096, False)
    expect = torch.cat([src[i * 1024:(i + 1) * 1024] for i in idx])
    assert torch.equal(dst, expect)
    back = torch.zeros_like(src)
    lib.ring_gather(0, back.data_ptr(), dst.data_ptr(), idx, 4096, True)
    for i in idx:
        assert torch.equal(back[i * 1024:(i + 1) * 1024], src[i * 1024:(i + 1) * 1024])
    m = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    lib.ring_memset(0, 4, m.data_ptr(), 0x7F7F7F7F, m.numel() * 4)
    assert bool((m == 0x7F7F7F7F).all())


def test_managed_gather_records_faults(gpu_rt):
    rows, dim = 4096, 1024  # bf16 rows of 2 KB
    b = rt.malloc_managed(rows * dim * 2, "emb")
    ref = torch.randn(rows, dim, dtype=torch.bfloat16)
    b.write(ref)
    idx = torch.tensor([0, 5, 1000, 4095, 2048], dtype=torch.int64, device="cuda")
    out = torch.empty(len(idx), dim, dtype=torch.bfloat16, device="cuda")
    lib.managed_gather(b.id, idx.data_ptr(), len(idx), dim * 2, out.data_ptr(), 0,
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref[idx.cpu()])
    n = lib.poll_device_faults(0)
    assert n == len(idx)
    assert lib.stats()["access_counter_notifications"] == len(idx)
    b.free()


def test_managed_gather_faults_attributed_to_channel(gpu_rt):
    """A stream registered as a user channel: the records k_managed_gather
    writes from it carry the channel, the service counts them per channel."""
    rows, dim = 1024, 1024
    b = rt.malloc_managed(rows * dim * 2, "emb-ch")
    b.write(torch.randn(rows, dim, dtype=torch.bfloat16))
    s = torch.cuda.Stream()
    cid = lib.register_channel(0, s.cuda_stream, "gather-stream")
    idx = torch.tensor([1, 2, 3], dtype=torch.int64, device="cuda")
    out = torch.empty(3, dim, dtype=torch.bfloat16, device="cuda")
    torch.cuda.synchronize()
    lib.managed_gather(b.id, idx.data_ptr(), 3, dim * 2, out.data_ptr(), 0, s.cuda_stream)
    s.synchronize()
    assert lib.poll_device_faults(0) == 3
    ch = [c for c in lib.channels() if c["id"] == cid][0]
    assert ch["remote_accesses"] == 3 and ch["error"] == "OK"
    lib.unregister_channel(cid)
    b.free()


def test_cxl_dma_roundtrip(gpu_rt):
    from ogkm import cxl

    buf = cxl.CxlBuffer.allocate(8 * MB)
    g = torch.arange(2 * MB, dtype=torch.int32, device="cuda")
    cxl.wait(buf.dma(g.data_ptr(), 0, 0, 8 * MB, cxl.DIR_GPU_TO_CXL))
    h = torch.zeros(2 * MB, dtype=torch.int32, device="cuda")
    cxl.wait(buf.dma(h.data_ptr(), 0, 0, 8 * MB, cxl.DIR_CXL_TO_GPU))
    assert torch.equal(g, h)
    buf.unregister()


def test_cxl_dma_full_rate_every_node(gpu_rt):
    """HBM <-> CXL pool on every NUMA node (local and the other socket) runs at
    the PCIe rate through a full-rate SDMA engine: the CXL ring used to pick an
    xGMI engine that moves GPU->host at 12.8 GB/s (profiles/r3_cxl_paths.md)."""
    import glob
    from ogkm import cxl

    nodes = sorted(int(p.rsplit("node", 1)[1]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
    lib.cxl_rediscover(-1, "/sys", sum(1 << n for n in nodes))
    res = {}
    for n in nodes:
        r = cxl.measure_bandwidth(0, 512 * MB, iters=3, node=n)
        res[n] = (round(r["gpu_to_cxl_gbps"], 1), round(r["cxl_to_gpu_gbps"], 1))
    print("hbm<->cxl per node (d2c, c2d) GB/s:", res, "gpu node", lib.device_numa_node(0))
    for n, (d2c, c2d) in res.items():
        assert d2c > 40 and c2d > 40, res


def test_ring_copy_bandwidth_d2h(gpu_rt):
    """GPU -> host through the D2H ring's SDMA engine at the PCIe rate."""
    n = 1 << 30
    g = torch.empty(n, dtype=torch.uint8, device="cuda")
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    lib.ring_copy(0, 1, h.data_ptr(), g.data_ptr(), n, True)
    t0 = time.perf_counter()
    for _ in range(3):
        lib.ring_copy(0, 1, h.data_ptr(), g.data_ptr(), n, True)
    gbps = 3 * n / (time.perf_counter() - t0) / 1e9
    print(f"D2H ring 1 GiB: {gbps:.1f} GB/s")
    assert gbps > 50


def test_peer_topology_on_hardware(gpu_rt):
    """parallel/topology.py on the real box (round 2 only ran it on fake
    devices): link types, NUMA node from sysfs, per-pair caps, CXL caps."""
    from ogkm.parallel import topology

    t = topology.discover()
    assert t.n >= 1 and t.link_name(0, 0) == "self"
    assert t.numa[0] == lib.device_numa_node(0) and t.numa[0] >= 0
    caps = t.p2p_caps(0, 0)
    assert caps["link"] == "self" and "cxl_reachable" in caps
    d = t.to_dict()
    print("topology", d)
    for a in range(t.n):
        for b in range(t.n):
            if a != b:
                assert t.link_name(a, b) in ("xgmi", "pcie")


def test_dmabuf_export(gpu_rt):
    b = rt.alloc_device_p2p(4 * MB, 0, "p2p")
    info = lib.range_info(b.id)
    fd, off = lib.export_dmabuf(info["ext_ptr"], 4 * MB)
    assert fd > 0
    os.close(fd)
    b.free()


def test_stable_va_vmm(gpu_rt):
    lib.configure("hbm_provider", 1)
    lib.init_device(0, 64 * MB)
    n = 6 * MB
    b = rt.malloc_managed(n, "stable", stable_va=True, device=0)
    ref = torch.arange(n // 4, dtype=torch.int32)
    b.write(ref)
    b.migrate("gpu:0")
    t = rt._tensor_from_ptr(b.dev_va, (n // 4,), torch.int32, "cuda", 0, b.id)
    assert torch.equal(t.cpu(), ref)
    del t
    b.free()


def test_stable_va_after_arena_recreation_reads_new_chunks(gpu_rt):
    """Re-creating the HBM arena releases its VMM handles together with the
    ROCr handles cached for stable-VA remaps (backend_hip.cpp vmm_release): a
    stable VA mapped in the new arena must read the new physical chunks, even
    when hipMemCreate hands back the same handle values. Each generation fills
    a different pattern, so a mapping to the old (leaked) memory shows up."""
    lib.configure("hbm_provider", 1)
    n = 6 * MB
    for gen in range(3):
        lib.init_device(0, 64 * MB)  # a fresh arena (the previous one is released)
        b = rt.malloc_managed(n, f"gen{gen}", stable_va=True, device=0)
        ref = torch.arange(n // 4, dtype=torch.int32) * (gen + 3) + 7 * gen
        b.write(ref)
        b.migrate("gpu:0")
        t = rt._tensor_from_ptr(b.dev_va, (n // 4,), torch.int32, "cuda", 0, b.id)
        assert torch.equal(t.cpu(), ref), f"generation {gen} reads stale memory"
        del t
        b.free()


def test_device_health_reports_ras_counters(gpu_rt):
    """ECC / xGMI RAS counters of the real GPU (amdgpu sysfs ras/aca_<block> or
    ras/<block>_err_count, else amd-smi): baselined at init, and a healthy box
    stays OK after a migration round trip. Unreadable counters are a reported
    condition with a reason, never a silent "healthy"
    (uvm_gpu.c:1328-1354, 2087-2104)."""
    buf = rt.malloc_managed(8 * MB, "health")
    buf.write(torch.arange(2 * MB, dtype=torch.int32))
    buf.migrate("gpu:0")
    buf.migrate("host")
    h = lib.device_health(0)
    print("device_health", h)
    assert h["status"] == "OK"
    assert h["reported"], h["unreadable_reason"]
    src = h["now"]["source"]
    assert src.startswith("sysfs:") or src == "amdsmi", src
    assert h["now"]["ue"] >= 0 and h["baseline"]["ue"] >= 0
    assert h["now"]["link_ue"] >= 0  # the xGMI (WAFL) block is read too
    buf.free()


def test_pluggable_allocator_subprocess():
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import torch, ogkm\n"
        "from ogkm import rt, allocator\n"
        "rt.init('hip', hbm_budget={0: 1<<30})\n"
        "allocator.enable()\n"
        "x = torch.randn(1024, 1024, device='cuda'); y = x @ x; torch.cuda.synchronize()\n"
        "s = allocator.stats(0); assert s['allocated'] > 0, s\n"
        "del x, y\n"
        "print('ALLOC_OK', s)\n"
    ) % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert "ALLOC_OK" in r.stdout, r.stdout + r.stderr


def test_managed_allocator_tensors_oversubscribe_subprocess():
    """Managed mode: 512 MB of torch tensors on a 256 MB arena. Parked tensors
    are evicted to host DRAM and come back at the same address with their
    contents when unparked; kernels on the current stream see the data."""
    code = (
        "import sys, time; sys.path.insert(0, %r)\n"
        "import torch, ogkm\n"
        "from ogkm import rt, allocator\n"
        "allocator.enable(managed_min_mb=4)\n"
        "rt.init('hip', hbm_budget={0: 256 << 20})\n"
        "xs = []\n"
        "for i in range(8):\n"
        "    x = torch.full((16 << 20,), float(i), device='cuda')\n"
        "    allocator.park(x); xs.append(x)\n"
        "torch.cuda.synchronize()\n"
        "s = allocator.managed_stats(0); assert s['parked_bytes'] == 8 * (64 << 20), s\n"
        "addrs = [x.data_ptr() for x in xs]\n"
        "t0 = time.perf_counter()\n"
        "for i, x in enumerate(xs):\n"
        "    allocator.unpark(x)\n"
        "    y = x * 2\n"
        "    assert bool((y == 2 * i).all()), i\n"
        "    del y\n"
        "    allocator.park(x)\n"
        "torch.cuda.synchronize()\n"
        "dt = time.perf_counter() - t0\n"
        "assert [x.data_ptr() for x in xs] == addrs\n"
        "ev = rt.stats()['evictions']; assert ev > 0, ev\n"
        "print('MANAGED_OK', allocator.managed_stats(0), 'evictions', ev, 'loop GB/s (host sync per tensor; throughput: next test)', 8 * 64 / 1024 / dt)\n"
    ) % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    print(r.stdout[-400:])
    assert "MANAGED_OK" in r.stdout, r.stdout + r.stderr


def test_managed_park_unpark_round_trip_throughput_subprocess():
    """Managed-tensor round-trip rate with the working set at 2x the arena
    (tools/bench_managed.py: 8 x 256 MB tensors, 1 GB arena, every touch brings
    256 MB in over PCIe and pushes another 256 MB out). Round 3 measured
    41-47 GB/s of touched bytes; the guard sits ~10% under the low end at 38 GB/s."""
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "bench_managed.py")
    r = subprocess.run([sys.executable, tool, "--tensors", "8", "--mb", "256", "--arena-mb", "1024", "--iters", "2"],
                       capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout + r.stderr
    res = json.loads(line[-1])
    print(res)
    assert res["correct"], res
    assert res["counters"].get("evictions", 0) > 0, res
    assert res["round_trip_gbps"] > 38.0, res


def test_allocator_free_on_busy_stream_is_stream_ordered(gpu_rt):
    """Free while the freeing stream is still busy writing the memory, then
    reallocate it on another stream: the new owner's write must land after the
    old one (the allocating stream waits GPU-side for the free's fence)."""
    n = 64 * MB
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    p = lib.torch_alloc(n, 0, s1.cuda_stream)
    old = rt._tensor_from_ptr(p, (n // 4,), torch.int32, "cuda", 0)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(200_000_000)     # keep s1 busy (~100 ms)
        old.fill_(1)
    lib.torch_free(p, 0, s1.cuda_stream)   # s1 has not run the fill yet
    q = lib.torch_alloc(n, 0, s2.cuda_stream)
    assert q == p                          # the same HBM comes back at once
    new = rt._tensor_from_ptr(q, (n // 4,), torch.int32, "cuda", 0)
    with torch.cuda.stream(s2):
        new.fill_(2)
    torch.cuda.synchronize()
    assert bool((new == 2).all())          # not overwritten by the old owner's late fill
    assert lib.torch_alloc_stats(0)[3] >= 1
    lib.torch_free(q, 0, s2.cuda_stream)


def test_allocator_same_stream_reuse_needs_no_wait(gpu_rt):
    """Freed and reallocated on the same stream: stream order already serialises
    the old and new owner, so no GPU-side wait is queued (and the data is right)."""
    n = 64 * MB
    s1 = torch.cuda.Stream()
    p = lib.torch_alloc(n, 0, s1.cuda_stream)
    old = rt._tensor_from_ptr(p, (n // 4,), torch.int32, "cuda", 0)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(100_000_000)
        old.fill_(1)
    waits0 = lib.torch_alloc_stats(0)[3]
    lib.torch_free(p, 0, s1.cuda_stream)
    q = lib.torch_alloc(n, 0, s1.cuda_stream)
    assert q == p and lib.torch_alloc_stats(0)[3] == waits0
    new = rt._tensor_from_ptr(q, (n // 4,), torch.int32, "cuda", 0)
    with torch.cuda.stream(s1):
        new.fill_(2)
    torch.cuda.synchronize()
    assert bool((new == 2).all())
    lib.torch_free(q, 0, s1.cuda_stream)


def test_allocator_small_slots_lazy_fences(gpu_rt):
    """Slab slots (<= 1 MB): a free records no event; reuse on the freeing
    stream records none either (stream order suffices), reuse from another
    stream records the fence then - on the freeing stream, so the new owner
    still runs after the old owner's late kernel."""
    n = 256 << 10
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    st0 = lib.torch_alloc_stats(0)
    ptrs = [lib.torch_alloc(n, 0, s1.cuda_stream) for _ in range(8)]  # one 2 MB slab
    for p in ptrs:
        lib.torch_free(p, 0, s1.cuda_stream)  # (the empty slab stays cached)
    again = [lib.torch_alloc(n, 0, s1.cuda_stream) for _ in range(8)]
    assert sorted(again) == sorted(ptrs)
    st1 = lib.torch_alloc_stats(0)
    assert st1[4] == st0[4] and st1[3] == st0[3], (st0, st1)  # no fence, no wait
    # cross-stream: the old owner is still queued behind a sleep on s1
    p = again[0]
    old = rt._tensor_from_ptr(p, (n // 4,), torch.int32, "cuda", 0)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(200_000_000)
        old.fill_(1)
    lib.torch_free(p, 0, s1.cuda_stream)
    q = lib.torch_alloc(n, 0, s2.cuda_stream)
    assert q == p
    new = rt._tensor_from_ptr(q, (n // 4,), torch.int32, "cuda", 0)
    with torch.cuda.stream(s2):
        new.fill_(2)
    torch.cuda.synchronize()
    assert bool((new == 2).all())
    st2 = lib.torch_alloc_stats(0)
    assert st2[4] == st1[4] + 1 and st2[3] >= st1[3] + 1, (st1, st2)
    lib.torch_free(q, 0, s2.cuda_stream)
    for x in again[1:]:
        lib.torch_free(x, 0, s1.cuda_stream)


def test_bf12_packed_stream_is_bit_exact(gpu_rt):
    """Fused H2D copy + BF12 decode kernel reproduces every bf16 bit pattern."""
    n = 5 * (1 << 20) + 4096  # 2.5 blocks, partial last block
    ref = (torch.randn(n // 2) * 0.02).to(torch.bfloat16)
    specials = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 3.0e38, 1e-40, -2.5, 1.0],
                            dtype=torch.bfloat16)
    ref[:len(specials)] = specials
    ref[-len(specials):] = specials
    b = rt.malloc_managed(n, "packed", packed_bf16=True)
    b.write(ref.cuda())
    res = b.residency(0)["resident_on"][0]
    assert res["tier"] == "host" and res["encoded_bytes"] < 0.8 * 2 * MB
    htd0 = lib.stats()["bytes_xfer_htd"]
    with b.acquire(0, rt.READ) as l:
        t = l.tensor((n // 2,), torch.bfloat16)
        torch.cuda.synchronize()
        assert torch.equal(t.view(torch.int16).cpu(), ref.view(torch.int16))
    s = lib.stats()
    assert s["decoded_bytes"] == n and s["bytes_xfer_htd"] - htd0 < 0.8 * n
    b.free()


def _refill_gbps(buf, n: int, reps: int = 3) -> float:
    """Best-of-`reps` rate (bf16 bytes delivered / s) of a host -> HBM refill of
    `buf`'s `n` bytes through the H2D ring (acquire of an evicted buffer)."""
    best = 0.0
    for _ in range(reps):
        buf.evict("gpu:0")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        l = buf.acquire(0, rt.READ)
        l.wait(0)
        dt = time.perf_counter() - t0
        l.release()
        best = max(best, n / dt / 1e9)
    return best


def test_bf12_decode_bandwidth(gpu_rt):
    """Packed streaming must deliver more bf16 bytes/s than the raw PCIe copy of
    the same GiB on the same box: a same-process ratio of best-of-3 refills,
    not an absolute number of one (round 5's driver box measured a single
    acquire at 43 GB/s). The default path is the fused copy + decode kernel;
    the SDMA-staged path (bf12_stage=1) is measured alongside for the record -
    it varies between processes (41-73 GB/s, profiles/r6_bf12_refill.md)."""
    lib.init_device(0, 3 << 30)
    n = 1 << 30
    data = (torch.randn(n // 2, device="cuda") * 0.02).to(torch.bfloat16)
    raw = rt.malloc_managed(n, "raw")
    raw.write(data)
    raw.set_read_mostly(True)
    raw_gbps = _refill_gbps(raw, n)
    raw.free()
    b = rt.malloc_managed(n, "pk", packed_bf16=True)
    b.write(data)
    b.set_read_mostly(True)
    gbps = _refill_gbps(b, n)  # default: the fused copy + decode kernel
    rt.configure(bf12_stage=1)  # for the record: SDMA staging + HBM decode
    s0 = lib.stats()
    staged = _refill_gbps(b, n, reps=2)
    s1 = lib.stats()
    rt.configure(bf12_stage=0)
    ring = {k: s1[k] - s0[k] for k in ("ring_copy_ns", "ring_copy_calls", "ring_idle_ns")}
    print(f"refill 1 GiB: raw {raw_gbps:.1f} GB/s, packed BF12 fused {gbps:.1f}, staged {staged:.1f} GB/s of bf16; "
          f"gpu numa {lib.device_numa_node(0)} host node {lib.host_node()}; staged ring {ring}")
    assert s1["packed_decodes"] > s0["packed_decodes"]  # the staged path ran
    # BF12 moves 0.75x the bytes: the ideal ratio is 1.33; guard at 90% of it
    # (measured 73.3 vs 57.1 GB/s = 1.28)
    assert gbps >= 1.2 * raw_gbps, (gbps, raw_gbps, staged)
    b.free()


@pytest.mark.parametrize("fmt,max_ratio,min_gbps", [("bf12", 0.78, 1000), ("bf11", 0.71, 1000), ("ans", 0.69, 800)])
def test_bf12_stream_unpack_hbm_bit_exact_and_fast(gpu_rt, fmt, max_ratio, min_gbps):
    """k_bf12_unpack (HBM-resident packed weights -> bf16 staging) reproduces every
    bit and runs at HBM speed (a 70B layer is ~1.7 GB of bf16), for BF12 and
    BF11 chunks (the kernel dispatches per chunk)."""
    from ogkm.ops import bf12

    n = (48 << 20) + 4096 + 6  # odd tail -> last chunk raw
    ref = (torch.randn(n) * 0.02).to(torch.bfloat16)
    specials = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 3.0e38, 1e-40, -2.5, 1.0],
                            dtype=torch.bfloat16)
    ref[:len(specials)] = specials
    ref[123457:123457 + len(specials)] = specials
    # exceptions in several tiles + a chunk of uniformly random bits (stored raw / BF12; ANS: every
    # exponent is a symbol, the random chunk is stored raw)
    ref[(5 << 20) + 17] = torch.tensor(1e30, dtype=torch.bfloat16)
    ref[(9 << 20) + 40000] = torch.tensor(-1e-30, dtype=torch.bfloat16)
    ref[(12 << 20):(13 << 20)] = torch.randint(-32768, 32767, (1 << 20,), dtype=torch.int16).view(torch.bfloat16)
    stream, info = bf12.pack(ref, fmt=fmt)
    assert info.ratio < max_ratio
    src = stream.cuda()
    dst = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    bf12.unpack_into(dst, src.data_ptr(), info, 0)
    torch.cuda.synchronize()
    assert torch.equal(dst.view(torch.int16).cpu(), ref.view(torch.int16))
    # bandwidth: bf16 bytes delivered per second
    for _ in range(3):
        bf12.unpack_into(dst, src.data_ptr(), info, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters = 20
    for _ in range(iters):
        bf12.unpack_into(dst, src.data_ptr(), info, 0)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    gbps = n * 2 / dt / 1e9
    print(f"{fmt} HBM unpack: {gbps:.0f} GB/s of bf16 written ({(info.nbytes + 2 * n) / dt / 1e9:.0f} GB/s HBM traffic)")
    assert gbps > min_gbps


def test_ans_unpack_reports_corrupt_chunk(gpu_rt):
    """A chunk whose ANS frequency table is not a valid distribution (zeroed here)
    is zero-filled and reported through lib.decode_errors() - the decoder never
    spins on it (before round 2 such a chunk cost a ~47 s decode-table scan)."""
    import struct

    from ogkm._native import lib
    from ogkm.ops import bf12

    n = 3 << 20
    ref = (torch.randn(n) * 0.02).to(torch.bfloat16)
    stream, info = bf12.pack(ref, fmt="ans")
    assert bf12.chunk_kinds(stream) == {3}
    off = struct.unpack_from("<Q", bytes(stream[32 + 16:32 + 24].numpy()))[0]  # chunk 1 payload
    bad = stream.clone()
    bad[off + 512:off + 1024] = 0  # u16 freq[256]
    src = bad.cuda()
    dst = torch.full((n,), 7.0, dtype=torch.bfloat16, device="cuda")
    lib.decode_errors(True)
    t0 = time.perf_counter()
    bf12.unpack_into(dst, src.data_ptr(), info, 0)
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 5.0
    err = lib.decode_errors(True)
    assert err["count"] >= 1 and err["stream"] == src.data_ptr() and err["chunk"] == 1 and err["detail"] == 0
    got = dst.view(torch.int16).cpu()
    cv = info.chunk_values
    assert torch.equal(got[:cv], ref.view(torch.int16)[:cv])
    assert torch.equal(got[2 * cv:], ref.view(torch.int16)[2 * cv:])
    assert (got[cv:2 * cv] == 0).all()


def test_fragmented_block_copy_page_list_kernel_gpu(gpu_rt):
    """Scattered pages of a host block -> HBM through one k_page_copy_lds
    launch (global_load_lds staging), bit-exact."""
    lib.configure("perf_prefetch_enable", 0)
    b = rt.malloc_managed(4 * MB, "frag")
    ref = _rand_bytes(4 * MB, seed=3)
    b.write(ref)
    pages = [p for p in range(1024) if p % 5 in (0, 2)]
    lib.service_faults([(b.id, p * 4096, 4096, 0, rt.READ) for p in pages])
    assert lib.stats()["page_list_copies"] >= 2          # one per block
    l = b.acquire(0, rt.READ)
    l.wait()
    t = l.tensor((4 * MB,), torch.uint8)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), ref)
    l.release()
    b.free()
