"""Packed host copies of read-mostly managed blocks (csrc/core/packer.cpp).

A block whose HBM copy keeps being dropped clean (or a SET_READ_MOSTLY one)
gets its host copy rewritten as one lossless ANS1 chunk; H2D refills then move
the packed bytes and the ring decodes them (DECODE_ANS). Fake backend: the
decode is the CPU reference codec, the protocol (eligibility, snapshot /
compare / install, expansion on writes and CPU access, whole-block sources) is
the runtime's own. The GPU twin (k_ans_blocks through the SDMA staging path)
is tests/test_packing_gpu.py."""
from __future__ import annotations

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20


def _weights(nbytes: int, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(nbytes // 2, generator=g) * 0.02).to(torch.bfloat16).view(torch.uint8)


def _packed_entries(b):
    out = []
    for off in range(0, b.size, 2 * MB):
        for e in b.residency(off)["resident_on"]:
            if e.get("encoded_bytes"):
                out.append((off, e["tier"], e["encoded_bytes"]))
    return out


def _pack(b) -> None:
    """READ_MOSTLY + one GPU read duplicate dropped clean: packed."""
    b.set_read_mostly(True)
    l = b.acquire(0, rt.READ)
    l.wait(0)
    l.release(0)
    b.evict("gpu:0")
    assert lib.pack_wait(30000)


def _gpu_read(b, dev=0, allow_remote=True) -> torch.Tensor:
    l = b.acquire(dev, rt.READ, allow_remote=allow_remote)
    l.wait(0)
    t = l.tensor((b.size,), torch.uint8).clone()
    l.release(0)
    return t


def test_read_mostly_block_packs_and_decodes_bit_exact(fake_rt):
    rt.configure(pack_host_copies=1, pack_threads=2)
    b = rt.malloc_managed(8 * MB, "w")
    data = _weights(b.size)
    b.write(data)
    b.set_read_mostly(True)
    assert lib.pack_wait(1000) and _packed_entries(b) == []  # the advice alone packs nothing
    _pack(b)
    packed = _packed_entries(b)
    assert len(packed) == 4 and all(t == "host" for _, t, _ in packed)
    ratio = sum(e for _, _, e in packed) / b.size
    assert 0.5 < ratio < 0.8, ratio  # exponent entropy of N(0, 0.02) bf16
    s0 = lib.stats()
    assert _gpu_read(b).equal(data)  # the H2D decoded the packed blocks
    s1 = lib.stats()
    assert s1["packed_decodes"] - s0["packed_decodes"] == 4
    # only the packed bytes crossed the link
    assert s1["bytes_xfer_htd"] - s0["bytes_xfer_htd"] == sum(e for _, _, e in packed)
    # read() and the CPU view see the raw data
    assert b.read().equal(data)
    st = lib.pack_stats()
    assert st["packed_blocks"] == 4 and st["queued"] == 0
    b.free()


def test_clean_evictions_trigger_packing(fake_rt):
    rt.configure(pack_host_copies=1, pack_threads=1, pack_auto_clean_evictions=2)
    b = rt.malloc_managed(4 * MB, "auto")
    data = _weights(b.size, 1)
    b.write(data)
    # accessed_by + a caller that needs the data at its own address (the
    # transparent mode's op holds): each read is a local read duplicate
    b.set_accessed_by(0)
    for _ in range(3):
        assert _gpu_read(b, allow_remote=False).equal(data)
        b.evict("gpu:0")  # a read duplicate: dropped without a copy-out
        lib.pack_wait(30000)
    assert len(_packed_entries(b)) == 2
    assert lib.stats()["packed_blocks"] == 2
    assert _gpu_read(b, allow_remote=False).equal(data)
    b.free()


def test_cpu_write_expands_packed_copy(fake_rt):
    rt.configure(pack_host_copies=1, pack_threads=1)
    b = rt.malloc_managed(4 * MB, "cw")
    data = _weights(b.size, 2)
    b.write(data)
    _pack(b)
    assert len(_packed_entries(b)) == 2
    # a CPU store through the CPU view: the packed copy is never mapped, so it
    # faults, expands (raw pages) and lands
    v = b.cpu_view()
    v[100] = 7
    data[100] = 7
    assert lib.stats()["pack_expansions"] >= 1
    assert b.read().equal(data)
    assert _gpu_read(b).equal(data)
    # a runtime write into the other block expands that one too
    patch = torch.full((4096,), 3, dtype=torch.uint8)
    b.write(patch, 3 * MB)
    data[3 * MB:3 * MB + 4096] = 3
    assert b.read().equal(data)
    assert _gpu_read(b).equal(data)
    b.free()


def test_gpu_write_revokes_and_source_expands(fake_rt):
    rt.configure(pack_host_copies=1, pack_threads=1)
    b = rt.malloc_managed(2 * MB, "gw")
    data = _weights(b.size, 3)
    b.write(data)
    _pack(b)
    assert len(_packed_entries(b)) == 1
    # a GPU write of one page revokes it in the packed host copy ...
    l = b.acquire(0, rt.WRITE, 8192, 4096)
    l.wait(0)
    l.tensor((4096,), torch.uint8).fill_(11)
    l.release(0)
    data[8192:12288] = 11
    # ... whose other pages still serve a refill of GPU 1 (expanded first: a
    # partial packed copy is no whole-block source)
    assert _gpu_read(b, 1).equal(data)
    assert b.read().equal(data)
    b.free()


def test_incompressible_blocks_stay_raw(fake_rt):
    rt.configure(pack_host_copies=1, pack_threads=1)
    b = rt.malloc_managed(2 * MB, "rand")
    data = torch.randint(0, 256, (b.size,), dtype=torch.uint8)
    b.write(data)
    _pack(b)
    assert _packed_entries(b) == []
    assert lib.stats()["pack_skips"] == 1
    assert _gpu_read(b).equal(data)
    b.free()


def test_packing_off_by_config(fake_rt):
    rt.configure(pack_host_copies=0)
    b = rt.malloc_managed(2 * MB, "off")
    b.write(_weights(b.size, 4))
    _pack(b)
    assert _packed_entries(b) == []
    b.free()


def test_packed_copy_moves_to_cxl_verbatim(fake_rt):
    """A packed host copy migrated down a tier moves its packed bytes as they
    are (no expansion) and still decodes bit-exact into HBM from there."""
    lib.cxl_rediscover(0, "/sys")  # emulate NUMA node 0 as a CXL pool
    rt.configure(pack_host_copies=1, pack_threads=1)
    b = rt.malloc_managed(2 * MB, "cxl")
    data = _weights(b.size, 5)
    b.write(data)
    _pack(b)
    assert len(_packed_entries(b)) == 1
    enc = _packed_entries(b)[0][2]
    s0 = lib.stats()
    b.migrate("cxl:0")  # (read-mostly: the host copy may stay as a duplicate)
    cxl = [e for _, t, e in _packed_entries(b) if t == "cxl"]
    assert cxl == [enc]
    assert lib.stats()["pack_expansions"] == s0["pack_expansions"]
    b.evict("host:0")
    assert _gpu_read(b).equal(data)
    b.free()


def test_written_block_goes_back_whole_without_expansion(fake_rt):
    """A GPU write into a block with a packed host copy: its eviction copies the
    whole block out raw over the packed copy (no host-side decode to merge the
    written pages), and the block is not packed again until it is dropped clean
    twice in a row."""
    rt.configure(pack_host_copies=1, pack_threads=1)
    b = rt.malloc_managed(2 * MB, "wb")
    data = _weights(b.size, 6)
    b.write(data)
    _pack(b)
    assert len(_packed_entries(b)) == 1
    l = b.acquire(0, rt.WRITE, 4096, 4096)
    l.wait(0)
    l.tensor((4096,), torch.uint8).fill_(9)
    l.release(0)
    data[4096:8192] = 9
    e0 = lib.stats()["pack_expansions"]
    b.evict("gpu:0")
    assert lib.stats()["pack_expansions"] == e0
    assert _packed_entries(b) == []
    assert lib.pack_wait(10000) and _packed_entries(b) == []  # written: not packed at once
    assert b.read().equal(data)
    assert _gpu_read(b).equal(data)
    b.free()


def test_staging_halves_rotate_under_many_packed_blocks(fake_rt):
    """More packed blocks than one staging half holds, in one refill: the ring
    alternates the halves (each refilled only after the decode that read it)
    and publishes the batch once its decodes completed."""
    rt.configure(pack_host_copies=1, pack_threads=2, ans_stage_mb=8)  # 2 x 4 MB halves: ~3 blocks each
    b = rt.malloc_managed(24 * MB, "many")
    data = _weights(b.size, 11)
    b.write(data)
    _pack(b)
    assert len(_packed_entries(b)) == 12
    s0 = lib.stats()
    for _ in range(3):
        assert _gpu_read(b).equal(data)
        b.evict("gpu:0")
    assert lib.stats()["packed_decodes"] - s0["packed_decodes"] == 36
    b.free()


def test_slow_decodes_never_race_chunk_reuse(fake_rt):
    """Packed-block decodes run behind the ring (their batch is published once
    they are done) while the next batches' copies go out: with a slow decode
    and an arena so small that just-decoded chunks are evicted and handed out
    again at once, every refill still reads back exactly (a copy into a chunk a
    decode still writes waits for that decode)."""
    rt.configure(pack_host_copies=1, pack_threads=2, fake_kernel_delay_us=3000)
    lib.init_device(0, 12 * MB)  # 6 chunks
    bufs, datas = [], []
    for i in range(6):
        b = rt.malloc_managed(4 * MB, f"s{i}")
        d = _weights(b.size, 20 + i) if i % 2 == 0 else torch.randint(0, 256, (4 * MB,), dtype=torch.uint8)
        b.write(d)
        b.set_read_mostly(True)
        bufs.append(b)
        datas.append(d)
    for b in bufs:  # one clean drop each: the bf16-like ones get packed
        l = b.acquire(0, rt.READ)
        l.wait(0)
        l.release(0)
        b.evict("gpu:0")
    assert lib.pack_wait(30000)
    assert sum(len(_packed_entries(b)) for b in bufs) == 6
    for rnd in range(4):
        # a burst of prefetches nobody waits for: each evicts the oldest
        # buffer's chunks - a packed one's decode may still be running there
        for b in bufs:
            b.prefetch("gpu:0")
        for i in (5, 4, 3):  # the three the burst left resident
            assert _gpu_read(bufs[i]).equal(datas[i]), (rnd, i)
    assert lib.stats()["packed_decodes"] > 0
    for b in bufs:
        b.free()


def test_queued_packed_batches_run_merged(fake_rt):
    """Refills of packed blocks queued behind a running batch run as ONE ring
    batch (ring_merge_packed_mb): fewer, fuller staging flushes; every buffer
    still reads back exactly and every tracking value is published."""
    rt.configure(pack_host_copies=1, pack_threads=2, fake_kernel_delay_us=2000, ring_merge_packed_mb=24)
    bufs, datas = [], []
    for i in range(8):
        b = rt.malloc_managed(4 * MB, f"m{i}")
        d = _weights(b.size, 40 + i)
        b.write(d)
        bufs.append(b)
        datas.append(d)
    for b in bufs:
        _pack(b)
    assert sum(len(_packed_entries(b)) for b in bufs) == 16
    s0 = lib.stats()
    for b in bufs:  # eight batches submitted back to back: the later ones queue
        b.prefetch("gpu:0")
    for b, d in zip(bufs, datas):
        assert _gpu_read(b).equal(d)
    s1 = lib.stats()
    assert s1["packed_decodes"] - s0["packed_decodes"] == 16
    assert s1["ring_merged_batches"] > s0["ring_merged_batches"]
    for b in bufs:
        b.free()


def test_block_leased_on_gpu_still_packs(fake_rt):
    """A block evicted clean and leased again on the GPU before the encoder
    reaches it (a hot block of a cyclic workload) still gets its host copy
    packed: the GPU lease never reads the host copy. Only a lease of the host
    copy itself defers the packing."""
    rt.configure(pack_host_copies=1, pack_threads=1)
    b = rt.malloc_managed(32 * MB, "hot")
    data = _weights(b.size, 77)
    b.write(data)
    b.set_read_mostly(True)
    l = b.acquire(0, rt.READ)
    l.wait(0)
    l.release(0)
    b.evict("gpu:0")  # 16 blocks queued for one encoder thread
    last = 30 * MB
    l = b.acquire(0, rt.READ, offset=last, length=2 * MB)  # the last block is back on the GPU, leased
    l.wait(0)
    assert lib.pack_wait(30000)
    assert any(o == last for o, _, _ in _packed_entries(b))
    t = l.tensor((2 * MB,), torch.uint8).clone()
    l.release(0)
    assert t.equal(data[last:last + 2 * MB])
    assert _gpu_read(b).equal(data)
    b.free()


@pytest.mark.parametrize("stage", [1, 0])
def test_bf12_refill_staged_and_fused_bit_exact(fake_rt, stage):
    """BF12-packed host copies refill HBM bit-exactly both through SDMA staging
    + HBM decode (bf12_stage=1, the default) and through the fused kernel that
    reads the host copy (bf12_stage=0); the staged path moves only encoded bytes."""
    fake_rt.configure(bf12_stage=stage)
    lib.init_device(0, 32 * MB)
    n = 6 * MB + 4096
    ref = (torch.randn(n // 2) * 0.02).to(torch.bfloat16)
    ref[:4] = torch.tensor([0.0, float("inf"), float("nan"), -2.5], dtype=torch.bfloat16)
    b = fake_rt.malloc_managed(n, "pk", packed_bf16=True)
    b.write(ref)
    for _ in range(2):
        b.evict("gpu:0")
        d0 = lib.stats()["packed_decodes"]
        with b.acquire(0, fake_rt.READ) as l:
            l.wait(0)
            got = l.tensor((n // 2,), torch.bfloat16).clone()  # the HBM copy the decode wrote
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
        if stage:
            assert lib.stats()["packed_decodes"] > d0
    b.free()


def _kv_step(b, data, pos):
    """One decode step of a KV-cache-like buffer, as the transparent mode runs
    it: the buffer leased on the GPU (a read duplicate of its host copy), ONE
    256 B entry written per 256 KB row, the written byte intervals revoking the
    other copies of just those pages (op-hold write invalidation), then evicted
    (only the written pages go back to the host copy)."""
    l = b.acquire(0, rt.READ)
    l.wait(0)
    t = l.tensor((b.size,), torch.uint8)
    assert t.equal(data)
    val = pos % 250 + 1
    spans = []
    for row in range(b.size // (256 << 10)):
        off = row * (256 << 10) + pos * 256
        t[off:off + 256] = val
        data[off:off + 256] = val
        spans.append((off, off + 256))
    lib.invalidate_others(b.id, spans, 0)
    l.release(0)
    b.evict("gpu:0")
    assert lib.pack_wait(30000)


def test_written_block_host_copy_packs_by_segment(fake_rt):
    """Page-granular packed residency for data written every step (a KV cache:
    one entry per row per step). The write-back marks the 64 KB segments it
    touched; the block's other segments pack (fmt 3: each segment its own ANS1
    chunk in a sidecar, written segments raw at their natural offsets). A
    refill decodes the packed segments and copies the raw ones; later writes
    into the same segments expand nothing, a write into a packed segment
    expands only that segment - and every read is bit-exact."""
    rt.configure(pack_host_copies=1, pack_segments=1, pack_threads=2)
    b = rt.malloc_managed(4 * MB, "kv")  # 2 blocks x 8 rows of 256 KB (4 segments per row)
    data = _weights(b.size, 21)
    b.write(data)
    b.set_read_mostly(True)
    _kv_step(b, data, 0)
    st = lib.pack_stats()
    assert st["seg_blocks"] == 2 and st["seg_packed"] == 2 * 24 and st["seg_raw"] == 2 * 8, st
    s0 = lib.stats()
    assert _gpu_read(b).equal(data)  # packed segments decoded, raw ones copied
    s1 = lib.stats()
    assert s1["seg_decodes"] - s0["seg_decodes"] == 48
    htd = s1["bytes_xfer_htd"] - s0["bytes_xfer_htd"]
    assert htd < 0.85 * b.size, htd  # 8 raw of 32 segments + ~0.68 of the 24 packed ones
    b.evict("gpu:0")
    e0 = lib.stats()["seg_expansions"]
    for pos in (1, 2, 3):  # the same (raw) segments: nothing expands, nothing re-packs
        _kv_step(b, data, pos)
    assert lib.stats()["seg_expansions"] == e0
    assert lib.pack_stats()["seg_packed"] == 48
    assert b.read().equal(data)
    # position 256 lies in each row's next segment, which rests packed: the
    # write-back decodes exactly those 16 segments; the cooled ones pack
    _kv_step(b, data, 256)
    assert lib.stats()["seg_expansions"] - e0 == 16
    assert lib.pack_stats()["seg_packed"] == 48
    assert b.read().equal(data)
    assert _gpu_read(b).equal(data)
    b.free()


def test_segmented_copy_cpu_access_and_runtime_write(fake_rt):
    """A runtime write into a packed segment expands that segment only; a CPU
    store through the CPU view faults (the view maps raw segments only) and
    the fault service - whole-block granular - expands the copy; all stay
    bit-exact through GPU refills."""
    rt.configure(pack_host_copies=1, pack_segments=1, pack_threads=1)
    b = rt.malloc_managed(2 * MB, "kv1")
    data = _weights(b.size, 22)
    b.write(data)
    b.set_read_mostly(True)
    _kv_step(b, data, 0)
    assert lib.pack_stats()["seg_packed"] == 24
    patch = torch.full((100,), 5, dtype=torch.uint8)
    b.write(patch, 70 * 1024)  # segment 1 (packed): expanded, then written
    data[70 * 1024:70 * 1024 + 100] = 5
    assert lib.pack_stats()["seg_packed"] == 23
    assert _gpu_read(b).equal(data)
    b.evict("gpu:0")
    v = b.cpu_view()
    v[3 * 65536 + 9] = 77  # CPU view store into packed segment 3
    data[3 * 65536 + 9] = 77
    assert lib.pack_stats()["seg_blocks"] == 0
    assert b.read().equal(data)
    assert _gpu_read(b).equal(data)
    b.free()
