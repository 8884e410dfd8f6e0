"""CXL tier tests - the fork's tests/cxl_p2p_test.c, rebuilt so they can fail on
data corruption (the reference's cannot: mismatches only print warnings)."""
from __future__ import annotations

import ctypes
import mmap

import pytest
import torch

from ogkm import cxl, rt
from ogkm._native import lib

MB = 1 << 20


def _fake_sysfs(tmp_path, with_cxl_bus=True):
    nodes = tmp_path / "devices" / "system" / "node"
    for nid, cpus, kb in ((0, "0-7", 1 << 20), (1, "8-15", 1 << 20), (2, "", 512 << 10)):
        d = nodes / f"node{nid}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
        (d / "meminfo").write_text(f"Node {nid} MemTotal:       {kb} kB\n")
        (d / "distance").write_text({0: "10 32 20", 1: "32 10 40", 2: "20 40 10"}[nid] + "\n")
    if with_cxl_bus:
        port = tmp_path / "bus" / "cxl" / "devices" / "port0"
        mem = tmp_path / "bus" / "cxl" / "devices" / "mem0"
        port.mkdir(parents=True)
        (mem / "ram").mkdir(parents=True)
        (mem / "ram" / "size").write_text(str(512 << 20))
        (mem / "numa_node").write_text("2")
        (tmp_path / "bus" / "cxl" / "devices" / "current_link_speed").write_text("32.0 GT/s PCIe")
        (tmp_path / "bus" / "cxl" / "devices" / "current_link_width").write_text("8")
    return tmp_path


def test_topology_from_sysfs(fake_rt, tmp_path):
    root = _fake_sysfs(tmp_path)
    info = cxl.rediscover(-1, str(root))
    assert info["numa_nodes"] == [2]
    assert info["memory_expander"] and info["link_up"] and not info["emulated"]
    assert info["cxl_version"] == 2  # Gen5 link
    assert any(d["name"] == "mem0" and d["numa_node"] == 2 for d in info["devices"])
    caps = cxl.p2p_caps(0, str(root))
    assert caps["connectivity"] == "CXL"
    # fake GPU 0 sits on node 0: the CXL node is 20 away (SLIT)
    assert caps["gpu_numa_node"] == 0 and caps["cxl_numa_distance"] == {2: 20} and caps["nearest_cxl_node"] == 2
    assert cxl.numa_distances(1, str(root)) == {0: 32, 1: 10, 2: 40}


def test_emulated_node(fake_rt, tmp_path):
    root = _fake_sysfs(tmp_path, with_cxl_bus=False)
    for p in (root / "devices" / "system" / "node" / "node2").iterdir():
        p.unlink()
    (root / "devices" / "system" / "node" / "node2").rmdir()
    info = cxl.rediscover(1, str(root))
    assert info["emulated"] and info["numa_nodes"] == [1]


def _buf(size):
    m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    return m, ctypes.addressof(ctypes.c_char.from_buffer(m))


def test_register_validation_and_unregister(fake_rt):
    m, base = _buf(8 * MB)
    with pytest.raises(rt.RuntimeStatusError):
        lib.cxl_register(base, 0, 2)          # size 0
    with pytest.raises(rt.RuntimeStatusError):
        lib.cxl_register(base, 8 * MB, 4)     # version must be 1..3
    with pytest.raises(rt.RuntimeStatusError):
        lib.cxl_register(base + 1, 4096, 2)   # unaligned
    h = lib.cxl_register(base, 8 * MB, 2)
    assert h >> 32 >= 1 and (h & 0xFFFFFFFF) >= 1   # opaque generation-checked handle
    with pytest.raises(rt.RuntimeStatusError, match="BUSY"):
        lib.cxl_register(base + 4 * MB, 4 * MB, 2)  # overlap
    info = lib.cxl_buffer(h)
    assert info["page_size"] in (4096, 2 * MB)
    assert info["backing_page"] >= 4096  # measured from /proc/self/smaps (hugetlbfs reports 2 MB / 1 GB)
    lib.cxl_unregister(h)
    with pytest.raises(rt.RuntimeStatusError, match="NOT_FOUND"):
        lib.cxl_unregister(h)               # stale handle
    h2 = lib.cxl_register(base, 8 * MB, 2)
    assert h2 != h                          # new generation
    lib.cxl_unregister(h2)


def test_buffer_limit_and_pin_budget(fake_rt):
    lib.shutdown()
    lib.config_reset()
    rt.init("fake", fake_devices=1, fake_hbm_mb=64, cxl_max_buffers=2)
    bufs = [_buf(2 * MB) for _ in range(3)]
    h = [lib.cxl_register(b, 2 * MB, 1) for _, b in bufs[:2]]
    with pytest.raises(rt.RuntimeStatusError, match="LIMIT_EXCEEDED"):
        lib.cxl_register(bufs[2][1], 2 * MB, 1)
    assert lib.cxl_info()["registered_buffers"] == 2
    assert lib.cxl_info()["pinned_bytes"] == 4 * MB
    for x in h:
        lib.cxl_unregister(x)
    assert lib.cxl_info()["pinned_bytes"] == 0


def test_pages_refcount_blocks_unregister(fake_rt):
    m, base = _buf(4 * MB)
    h = lib.cxl_register(base, 4 * MB, 3)
    ext = lib.cxl_pages(h, 4096, 3 * MB)
    assert sum(n for _, n in ext) == 3 * MB and ext[0][0] == base + 4096
    with pytest.raises(rt.RuntimeStatusError, match="BUSY"):
        lib.cxl_unregister(h)
    lib.cxl_put_pages(h)
    lib.cxl_unregister(h)


def test_dma_roundtrip_verifies_data(fake_rt):
    """GPU -> CXL then CXL -> GPU; any corruption fails the test."""
    buf = cxl.CxlBuffer.allocate(4 * MB)
    g = rt.malloc_managed(4 * MB, "g")
    lg = g.acquire(0, rt.WRITE)
    lg.wait(0)
    pattern = (torch.arange(4 * MB, dtype=torch.int64) + 0xAB).remainder(256).to(torch.uint8)
    lg.tensor((4 * MB,), torch.uint8).copy_(pattern)
    cxl.wait(buf.dma(lg.dptr, 0, 0, 4 * MB, cxl.DIR_GPU_TO_CXL))
    host = (ctypes.c_uint8 * (4 * MB)).from_address(buf.base)
    assert bytes(host[:16]) == bytes(pattern[:16].tolist())
    lg.tensor((4 * MB,), torch.uint8).zero_()
    tid = buf.dma(lg.dptr, 0, 0, 4 * MB, cxl.DIR_CXL_TO_GPU, async_=True)
    cxl.wait(tid)
    assert torch.equal(lg.tensor((4 * MB,), torch.uint8), pattern)
    with pytest.raises(rt.RuntimeStatusError):
        buf.dma(lg.dptr, 0, 2 * MB, 4 * MB, cxl.DIR_CXL_TO_GPU)  # out of bounds
    s = lib.stats()
    assert s["cxl_dma_requests"] == 2 and s["cxl_dma_bytes"] == 8 * MB
    lg.release(0)
    g.free()
    buf.unregister()


def _two_socket_sysfs(tmp_path):
    """Two CPU sockets (nodes 0, 1), each with a CPU-less CXL node attached:
    node 2 behind socket 1, node 3 behind socket 0 (ids deliberately crossed,
    so 'first node' and 'nearest node' differ for socket 0)."""
    nodes = tmp_path / "devices" / "system" / "node"
    slit = {0: "10 32 40 20", 1: "32 10 20 40", 2: "40 20 10 50", 3: "20 40 50 10"}
    for nid, cpus in ((0, "0-7"), (1, "8-15"), (2, ""), (3, "")):
        d = nodes / f"node{nid}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
        (d / "meminfo").write_text(f"Node {nid} MemTotal:       {1 << 20} kB\n")
        (d / "distance").write_text(slit[nid] + "\n")
    return tmp_path


def test_demotion_goes_to_nearest_cxl_node(fake_rt, tmp_path):
    """Host-tier data demotes to the CXL pool nearest the host node it leaves
    (block_select_node_residency, uvm_va_block.c:11714-11760), not to the first
    CXL node: socket 0 -> node 3, socket 1 -> node 2."""
    root = _two_socket_sysfs(tmp_path)
    info = cxl.rediscover(-1, str(root))
    assert info["numa_nodes"] == [2, 3]
    assert lib.cxl_nearest_node(0) == 3 and lib.cxl_nearest_node(1) == 2
    TIER_HOST, TIER_CXL = 1, 2
    assert lib.demotion_target(TIER_HOST, 0) == (TIER_CXL, 3)
    assert lib.demotion_target(TIER_HOST, 1) == (TIER_CXL, 2)
    # the demotions of a full host tier land on node 3 (nearest to host node 0)
    lib.configure("host_budget_mb", 8)
    lib.init_device(0, 8 * MB)
    bufs = []
    for i in range(6):
        b = rt.malloc_managed(4 * MB, f"d{i}")
        l = b.acquire(0, rt.WRITE)
        l.wait(0)
        l.tensor((4 * MB,), torch.uint8).fill_(i + 1)
        l.release(0)
        bufs.append(b)
    placed = [(r["tier"], r["id"]) for b in bufs for o in (0, 2 * MB) for r in b.residency(o)["resident_on"]]
    assert ("cxl", 3) in placed and ("cxl", 2) not in placed, placed
    for i, b in enumerate(bufs):
        assert int(b.read().min()) == i + 1
        b.free()


def test_emulated_cxl_pool_per_socket(fake_rt, tmp_path):
    """Without CXL hardware, one emulated pool per socket: a host node's own
    DRAM is never its CXL tier while another pool exists (the same memory
    would back both tiers), so each host node demotes to the other socket."""
    root = _two_socket_sysfs(tmp_path)
    for nid in (2, 3):  # drop the CPU-less nodes: a plain 2-socket box
        for f in (root / "devices" / "system" / "node" / f"node{nid}").iterdir():
            f.unlink()
        (root / "devices" / "system" / "node" / f"node{nid}").rmdir()
    for nid, row in ((0, "10 32"), (1, "32 10")):
        (root / "devices" / "system" / "node" / f"node{nid}" / "distance").write_text(row + "\n")
    info = cxl.rediscover(-1, str(root), emulate_nodes=(0, 1))
    assert info["emulated"] and info["numa_nodes"] == [0, 1]
    assert lib.cxl_nearest_node(0) == 1 and lib.cxl_nearest_node(1) == 0
    info = cxl.rediscover(-1, str(root), emulate_nodes=(1,))  # bench.py: the host node left out of the pool
    assert info["numa_nodes"] == [1] and lib.cxl_nearest_node(0) == 1
    info = cxl.rediscover(-1, str(root), emulate_nodes=(0,))  # single-node box: the only pool is the host's
    assert lib.cxl_nearest_node(0) == 0
