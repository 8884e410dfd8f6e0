"""Peer-memory client tests (fake backend): 64 KB page tables, pinning against
eviction, owner-free invalidation callbacks, persistent clients, dma-buf
export and cross-process IPC. Mirrors what nvidia-peermem / nvidia_p2p_* do
(pm/nvidia-peermem.c:129-300, kernel-open/nvidia/nv-p2p.c:362-942); the
reference has no automated test for these paths."""
from __future__ import annotations

import mmap
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from ogkm import p2p, rt
from ogkm._native import lib

MB = 1 << 20
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_page_table_and_sg_list(fake_rt):
    b = rt.malloc_managed(4 * MB, "p2p")
    b.write(torch.arange(MB, dtype=torch.int32))
    c = p2p.PeerMemClient()
    reg = c.get_pages(b, 64 << 10, 3 * MB, device=0)
    pages = reg.pages()
    assert len(pages) == 3 * MB // (64 << 10)
    assert all(pages[i + 1] - pages[i] == 64 << 10 for i in range(len(pages) - 1))
    assert reg.dma_map() == [(reg.dptr, 3 * MB)]
    # the pinned device copy holds the data
    t = reg.tensor((3 * MB // 4,), torch.int32)
    assert torch.equal(t[:8], torch.arange(16384, 16392, dtype=torch.int32))
    # misaligned offsets are refused like nv-p2p's 64 KB check
    with pytest.raises(ValueError):
        c.get_pages(b, 4096, MB)
    assert c.acquire(b, 0, MB, 0)
    assert not c.acquire(b, 4096, MB, 0)
    reg.put()
    assert not reg.valid and c.regions() == []
    c.close()
    b.free()


def test_pinned_region_survives_pressure(fake_rt):
    # 64 MB HBM per fake device: pin 8 MB, then stream 96 MB through device 0.
    b = rt.malloc_managed(8 * MB, "pinned")
    b.write(torch.full((2 * MB,), 7, dtype=torch.int32))
    c = p2p.PeerMemClient()
    reg = c.get_pages(b, 0, 8 * MB, 0)
    dptr = reg.dptr
    others = [rt.malloc_managed(16 * MB, f"o{i}") for i in range(6)]
    for o in others:
        o.fill(0x01010101)
        o.prefetch("gpu:0")
        lib.sync_all()
    # still resident at the same device address with the same data
    assert reg.dptr == dptr
    res = b.residency(0)
    assert ("gpu", 0) in [(r["tier"], r["id"]) for r in res["resident_on"]]
    assert int(reg.tensor((2 * MB,), torch.int32)[12345]) == 7
    reg.put()
    for o in others:
        o.free()
    c.close()
    b.free()


def test_free_invalidates_importer(fake_rt):
    b = rt.malloc_managed(2 * MB, "inv")
    c = p2p.PeerMemClient()
    seen = []
    reg = c.get_pages(b, 0, 2 * MB, 1, free_callback=lambda r: seen.append(r))
    b.free()  # owner frees while the importer still holds the region
    assert seen == [reg] and not reg.valid
    assert c.stats["invalidations"] == 1
    with pytest.raises(RuntimeError):
        reg.pages()
    c.close()


def test_persistent_client_blocks_free(fake_rt):
    b = rt.malloc_managed(2 * MB, "persist")
    c = p2p.PeerMemClient(persistent=True)
    reg = c.get_pages(b, 0, MB, 0)
    with pytest.raises(RuntimeError):
        b.free()
    reg.put()
    c.close()
    b.free()


def test_export_dmabuf_fd_maps_same_bytes(fake_rt):
    b = rt.alloc_device_p2p(4 * MB, 0, "exp")
    c = p2p.PeerMemClient()
    reg = c.get_pages(b, MB, 2 * MB, 0)
    reg.tensor((2 * MB,), torch.uint8).fill_(0x5A)
    fd, off = reg.export_dmabuf()
    try:
        m = mmap.mmap(fd, off + 2 * MB, mmap.MAP_SHARED, mmap.PROT_READ)
        assert m[off] == 0x5A and m[off + 2 * MB - 1] == 0x5A
        m.close()
    finally:
        os.close(fd)
    reg.put()
    c.close()
    b.free()


def test_ipc_cross_process(fake_rt):
    b = rt.malloc_managed(2 * MB, "ipc")
    b.write(torch.arange(MB // 2, dtype=torch.int32))
    c = p2p.PeerMemClient()
    reg = c.get_pages(b, 0, 2 * MB, 0)
    h = reg.ipc_handle()
    child = textwrap.dedent(f"""
        import sys, torch
        sys.path.insert(0, {ROOT!r})
        import ogkm
        from ogkm import rt, p2p
        rt.init("fake", fake_devices=2, fake_hbm_mb=64)
        with p2p.open_ipc(bytes.fromhex(sys.argv[1]), {2 * MB}) as m:
            t = m.tensor(({MB // 2},), torch.int32)
            ok = int(t[1000]) == 1000
            t[0] = 4242          # write through the peer mapping
        print("OK" if ok else "BAD")
    """)
    r = subprocess.run([sys.executable, "-c", child, h.hex()], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-2000:]
    assert int(reg.tensor((MB // 2,), torch.int32)[0]) == 4242
    reg.put()
    c.close()
    b.free()


def test_collective_timeout_sets_sticky_fatal():
    """A collective that fails (here: a peer that never joins, caught by the
    process-group timeout) raises comm.CollectiveError and sets the runtime's
    sticky FATAL status, so later runtime calls fail fast."""
    import json
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(root, "tests/helpers/comm_fault_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    line = [l for l in r.stdout.splitlines() if l.startswith("COMMFAULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads(line[0][len("COMMFAULT "):])
    assert out["raised"] and out["status"] == "FATAL" and "all_reduce_" in out["reason"]
    assert out["malloc_after"] != "ok" and "FATAL" in out["malloc_after"]


_IMPORTER = textwrap.dedent("""
    import sys, torch
    sys.path.insert(0, sys.argv[4])
    import ogkm
    from ogkm import rt, p2p
    backend = sys.argv[3]
    if backend == "fake":
        rt.init("fake", fake_devices=1, fake_hbm_mb=64)
    else:
        rt.init("hip", hbm_budget={0: 1 << 30})
    from ogkm._native import lib
    fd, off = int(sys.argv[1]), int(sys.argv[2])
    dev = "cpu" if backend == "fake" else "cuda"
    with p2p.DmabufImport(fd, 0) as imp:
        # The mapping is device-visible only (the HIP runtime does not track it):
        # move data with the runtime's copy kernels, not hipMemcpy.
        got = torch.zeros(1000, dtype=torch.int32, device=dev)
        lib.ring_copy(0, 2, got.data_ptr(), imp.ptr + off, 4000, True)
        ok = bool((got == torch.arange(1000, dtype=torch.int32, device=dev)).all())
        val = torch.tensor([-77], dtype=torch.int32, device=dev)
        lib.ring_copy(0, 2, imp.ptr + off + 20, val.data_ptr(), 4, True)  # write through the importer's mapping
    print("IMPORT_OK" if ok else "IMPORT_BAD", flush=True)
""")


def _dmabuf_round_trip(backend):
    b = rt.alloc_device_p2p(4 * MB, 0, "exp")
    info = lib.range_info(b.id)
    dev = "cpu" if backend == "fake" else "cuda"
    src = rt._tensor_from_ptr(info["ext_ptr"], (MB,), torch.int32, dev, 0)
    src.copy_(torch.arange(MB, dtype=torch.int32, device=dev))
    if backend != "fake":
        torch.cuda.synchronize()
    fd, off = lib.export_dmabuf(info["ext_ptr"], 4 * MB)
    r = subprocess.run([sys.executable, "-c", _IMPORTER, str(fd), str(off), backend, ROOT], pass_fds=(fd,),
                       capture_output=True, text=True, timeout=240)
    os.close(fd)
    assert r.returncode == 0 and "IMPORT_OK" in r.stdout, r.stdout + r.stderr[-2000:]
    assert int(src[5]) == -77                      # the importer's write is visible to the exporter
    b.free()


def test_dmabuf_import_cross_process(fake_rt):
    """Exporter (this process) -> dma-buf fd -> importer (another process) maps
    it, reads the exporter's data and writes back through its mapping."""
    _dmabuf_round_trip("fake")


@pytest.mark.gpu
def test_dmabuf_import_cross_process_gpu(gpu_rt):
    _dmabuf_round_trip("hip")
