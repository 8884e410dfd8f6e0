"""Packed host copies on the GPU (csrc/core/packer.cpp + Ring DECODE_ANS +
k_ans_blocks): a read-mostly managed buffer whose HBM copy was dropped clean is
packed on the host; its next H2D refill moves only the packed bytes - SDMA into
the ring's HBM staging buffer, then ONE k_ans_blocks launch per batch of
blocks (the default engine path) or k_ans_blocks reading the host copy
directly (CU copy-kernel rings) - and the HBM copy is bit-identical to the
data written. The CPU twin is tests/test_packing.py."""
from __future__ import annotations

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

pytestmark = pytest.mark.gpu

MB = 1 << 20


def _weights(nbytes: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(nbytes // 2, generator=g) * 0.02).to(torch.bfloat16).view(torch.uint8)


def _packed(b):
    out = []
    for off in range(0, b.size, 2 * MB):
        for e in b.residency(off)["resident_on"]:
            if e.get("encoded_bytes"):
                out.append(e["encoded_bytes"])
    return out


@pytest.mark.parametrize("engine", [3, 0], ids=["sdma_staging", "kernel_direct"])
def test_packed_refill_bit_exact(gpu_rt, engine):
    if engine != rt.get_config("copy_engine"):
        # the rings pick their engine path when they are created
        lib.shutdown()
        rt.init("hip", lock_check=1, host_budget_mb=16384, hbm_budget={0: 2 << 30}, copy_engine=engine)
    rt.configure(pack_host_copies=1, pack_threads=4)
    size = 96 * MB + 12 * 4096  # 48 full blocks + a partial last block
    b = rt.malloc_managed(size, "packed")
    data = _weights(size, 7)
    b.write(data)
    b.set_read_mostly(True)
    l = b.acquire(0, rt.READ)
    l.wait()
    l.release()
    b.evict("gpu:0")  # a clean read duplicate: the host copy gets packed
    assert lib.pack_wait(60000)
    enc = _packed(b)
    assert len(enc) == 49, len(enc)
    assert sum(enc) < 0.75 * size
    s0 = lib.stats()
    l = b.acquire(0, rt.READ)
    l.wait()
    got = l.tensor((size,), torch.uint8)
    ok = torch.equal(got, data.cuda())
    l.release()
    s1 = lib.stats()
    assert ok
    assert s1["packed_decodes"] - s0["packed_decodes"] == 49
    assert s1["bytes_xfer_htd"] - s0["bytes_xfer_htd"] == sum(enc)
    err = lib.decode_errors(True)
    assert err["count"] == 0, err
    # the host copy stays packed (a read duplicate) and serves again
    b.evict("gpu:0")
    l = b.acquire(0, rt.READ, 50 * MB, 8 * MB)
    l.wait()
    assert torch.equal(l.tensor((8 * MB,), torch.uint8), data[50 * MB:58 * MB].cuda())
    l.release()
    b.free()


def test_gpu_write_after_packing_round_trips(gpu_rt):
    """A GPU write into a packed block revokes the packed pages; the data comes
    back right through eviction (the write-back expands the host copy)."""
    rt.configure(pack_host_copies=1, pack_threads=2)
    b = rt.malloc_managed(8 * MB, "pw")
    data = _weights(b.size, 8)
    b.write(data)
    b.set_read_mostly(True)
    l = b.acquire(0, rt.READ)
    l.wait()
    l.release()
    b.evict("gpu:0")
    assert lib.pack_wait(60000) and len(_packed(b)) == 4
    l = b.acquire(0, rt.WRITE, 3 * MB, 4096)
    l.wait()
    l.tensor((4096,), torch.uint8).fill_(5)
    torch.cuda.synchronize()
    l.release()
    data[3 * MB:3 * MB + 4096] = 5
    b.evict("gpu:0")
    assert torch.equal(b.read(), data)
    l = b.acquire(0, rt.READ)
    l.wait()
    assert torch.equal(l.tensor((b.size,), torch.uint8), data.cuda())
    l.release()
    b.free()


@pytest.mark.parametrize("engine", [3, 0], ids=["sdma_staging", "kernel_direct"])
def test_segmented_kv_refill_bit_exact(gpu_rt, engine):
    """A KV-cache-like buffer written every step (one 256 B entry per 256 KB
    row, page-granular write invalidation as the transparent mode's op holds
    do): its host copy rests segment-packed (fmt 3) - 24 of every block's 32
    segments as ANS1 chunks, the written ones raw - and refills through the
    ring decode the packed segments (k_ans_blocks, one staging copy per block)
    and copy the raw ones, bit-exact every step, including the step whose
    writes move into packed segments."""
    if engine != rt.get_config("copy_engine"):
        lib.shutdown()
        rt.init("hip", lock_check=1, host_budget_mb=16384, hbm_budget={0: 2 << 30}, copy_engine=engine)
    rt.configure(pack_host_copies=1, pack_segments=1, pack_threads=4)
    size = 32 * MB
    b = rt.malloc_managed(size, "kv")
    data = _weights(size, 9).cuda()
    b.write(data)
    b.set_read_mostly(True)
    rows = size // (256 << 10)
    for step, pos in enumerate((0, 1, 2, 256, 257)):
        l = b.acquire(0, rt.READ)
        l.wait()
        t = l.tensor((size,), torch.uint8)
        assert torch.equal(t, data), (step, pos)
        spans = []
        val = pos % 250 + 1
        for row in range(rows):
            off = row * (256 << 10) + pos * 256
            t[off:off + 256] = val
            data[off:off + 256] = val
            spans.append((off, off + 256))
        torch.cuda.synchronize()
        lib.invalidate_others(b.id, spans, 0)
        l.release()
        b.evict("gpu:0")
        assert lib.pack_wait(60000)
        if step == 1:  # (step 0's eviction wrote the whole block: the data was written on the GPU)
            st = lib.pack_stats()
            assert st["seg_blocks"] == size // (2 * MB) and st["seg_packed"] == 24 * (size // (2 * MB)), st
    s0 = lib.stats()
    l = b.acquire(0, rt.READ)
    l.wait()
    assert torch.equal(l.tensor((size,), torch.uint8), data)
    l.release()
    s1 = lib.stats()
    assert s1["seg_decodes"] - s0["seg_decodes"] == 24 * (size // (2 * MB))
    assert s1["bytes_xfer_htd"] - s0["bytes_xfer_htd"] < 0.85 * size
    assert torch.equal(b.read().cuda(), data)
    b.free()


def test_single_segment_chunks_decode_one_wave_each(gpu_rt):
    """k_ans_segs (one wave per single-segment ANS1 chunk - the chunks of
    segmented host copies) decodes every bit, including special values and a
    corrupt chunk (reported and zero-filled, the others unaffected), and
    prints its throughput next to the 4-segment-item stream kernel (it is the
    slower one in bulk - see the guard)."""
    from ogkm.ops import bf12
    import time

    nseg = 2048  # 128 MB of bf16
    n = nseg * 32768
    ref = (torch.randn(n) * 0.02).to(torch.bfloat16)
    ref[:4] = torch.tensor([0.0, float("inf"), float("nan"), -2.5], dtype=torch.bfloat16)
    stream, info = bf12.pack(ref, chunk_values=32768, fmt="ans")
    assert info.nchunks == nseg
    table = stream[32:32 + 16 * nseg].view(torch.int32).view(-1, 4)  # {u64 offset, u32 n_values, u32 encoded}
    offs = [int(lo) & 0xFFFFFFFF | (int(hi) << 32) for lo, hi in table[:, :2].tolist()]
    kinds = table[:, 3].tolist()
    assert set(kinds) == {3}  # every chunk ANS1
    src = stream.cuda()
    dst = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    base = src.data_ptr()
    srcs = [base + o for o in offs]
    dsts = [dst.data_ptr() + 2 * 32768 * i for i in range(nseg)]
    nv = [32768] * nseg
    lib.decode_errors(True)
    lib.decode_ans_chunks(0, srcs, dsts, nv, 0)
    torch.cuda.synchronize()
    assert torch.equal(dst.view(torch.int16).cpu(), ref.view(torch.int16))
    for _ in range(2):
        lib.decode_ans_chunks(0, srcs, dsts, nv, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        lib.decode_ans_chunks(0, srcs, dsts, nv, 0)
    torch.cuda.synchronize()
    seg_gbps = 10 * 2 * n / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    for _ in range(10):
        bf12.unpack_into(dst, src.data_ptr(), info, 0)
    torch.cuda.synchronize()
    item_gbps = 10 * 2 * n / (time.perf_counter() - t0) / 1e9
    print(f"single-segment chunks: k_ans_segs {seg_gbps:.0f} GB/s, k_ans_unpack {item_gbps:.0f} GB/s of bf16")
    # k_ans_segs takes its descriptors inline (kAnsInlineSegs = 128 per launch:
    # 128 waves, a sliver of the chip, each decoding 32 Ki values serially), so
    # a bulk decode of 2048 chunks is 16 latency-bound launches - measured 67
    # GB/s against k_ans_unpack's ~960 (gpurun_out/r6/ae_suite.log). A refill
    # hands it at most one block's 32 segments per descriptor batch; the guard
    # only catches a broken or serialised kernel.
    assert seg_gbps > 30
    # a corrupt chunk: reported, zero-filled; its neighbours still decode
    bad = src.clone()
    bad[offs[5]:offs[5] + 4] = 0  # magic
    lib.decode_errors(True)
    lib.decode_ans_chunks(0, [bad.data_ptr() + o for o in offs[:8]], dsts[:8], nv[:8], 0)
    torch.cuda.synchronize()
    assert lib.decode_errors(True)["count"] >= 1
    got = dst[:8 * 32768].view(torch.int16).cpu()
    assert torch.equal(got[5 * 32768:6 * 32768], torch.zeros(32768, dtype=torch.int16))
    assert torch.equal(got[4 * 32768:5 * 32768], ref[4 * 32768:5 * 32768].view(torch.int16))
