"""Fused decode-step ops (csrc/kernels/decode_ops.hip; CPU references in
csrc/core/dgemm_ref.cpp) vs plain fp32 PyTorch: RMSNorm, RoPE + KV append,
GQA decode attention (flash-decoding split over the context)."""
from __future__ import annotations

import math

import pytest
import torch

from ogkm.ops import decode as D
from ogkm.ops import fused


def _dev(gpu):
    return "cuda" if gpu else "cpu"


def _check_rmsnorm(gpu, dim=1024):
    x = (torch.randn(5, dim) * 3).to(torch.bfloat16)
    w = (torch.rand(dim) + 0.5).to(torch.bfloat16)
    want = D.rms_norm(x.float(), w.float(), 1e-5)
    got = fused.rms_norm(x.to(_dev(gpu)), w.to(_dev(gpu)), 1e-5)
    torch.testing.assert_close(got.float().cpu(), want, atol=2e-2, rtol=2e-2)


def _check_rope_kv(gpu):
    B, hq, hkv, hd, T, pos = 3, 8, 2, 64, 40, 17
    qkv = torch.randn(B, (hq + 2 * hkv) * hd).to(torch.bfloat16)
    cos, sin = D.rope_tables(hd, T, 500000.0, "cpu")
    cache = torch.zeros(2, B, hkv, T, hd, dtype=torch.bfloat16)
    tail = torch.zeros(2, B, hkv, 4, hd, dtype=torch.bfloat16)
    dv = _dev(gpu)
    cd, td = cache.to(dv), tail.to(dv)
    q = fused.rope_kv(qkv.to(dv), cos[pos].to(dv), sin[pos].to(dv), cd, pos, hq, hkv, tail=td, tail_pos=2)
    qr = D.apply_rope(qkv[:, :hq * hd].view(B, hq, hd).float(), cos[pos], sin[pos])
    kr = D.apply_rope(qkv[:, hq * hd:(hq + hkv) * hd].view(B, hkv, hd).float(), cos[pos], sin[pos])
    v = qkv[:, (hq + hkv) * hd:].view(B, hkv, hd).float()
    torch.testing.assert_close(q.float().cpu(), qr, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(cd[0, :, :, pos].float().cpu(), kr, atol=2e-2, rtol=2e-2)
    assert torch.equal(cd[1, :, :, pos].cpu(), qkv[:, (hq + hkv) * hd:].view(B, hkv, hd))
    assert torch.equal(td[:, :, :, 2].cpu(), cd[:, :, :, pos].cpu())
    assert cd[:, :, :, pos + 1:].abs().sum() == 0 and cd[:, :, :, :pos].abs().sum() == 0


def _check_attention(gpu, length, hq=16, hkv=2, hd=128, split_tokens=0):
    B, T = 2, 700
    q = torch.randn(B, hq, hd).to(torch.bfloat16)
    cache = torch.randn(2, B, hkv, T, hd).to(torch.bfloat16)
    want = D.gqa_decode_attention(q.float(), cache[0].float(), cache[1].float(), length)
    dv = _dev(gpu)
    got = fused.attention(q.to(dv), cache.to(dv), length, split_tokens=split_tokens)
    torch.testing.assert_close(got.float().cpu(), want, atol=2e-2, rtol=2e-2)


def _check_deferred_epilogues(gpu, d=1024):
    """dgemm.linear(defer=True) + the consumer's fused epilogue == the separate
    reduce launch, bit for bit: residual add + RMSNorm (o / down projections)
    and the qkv store epilogue inside RoPE + KV append; a later linear() call
    invalidates the deferred partials (loud error, not stale data)."""
    from ogkm.ops import dgemm
    dv = _dev(gpu)
    m, k = 7, 2048
    g = torch.Generator().manual_seed(11)
    wt = (torch.randn(d, k, generator=g) * 0.02).to(torch.bfloat16)
    wbuf = dgemm.frag_permute(wt).contiguous().to(dv)
    wref = dgemm.WeightRef(wbuf.data_ptr(), 0, d, k, dgemm.MODE_RAW)
    a = (torch.randn(m, k, generator=g) * 0.5).to(torch.bfloat16).to(dv)
    x0 = (torch.randn(m, d, generator=g) * 0.3).to(torch.bfloat16).to(dv)
    nw = (torch.rand(d, generator=g) + 0.5).to(torch.bfloat16).to(dv)
    xa = x0.clone()
    dgemm.linear(a, wref, "resid", resid=xa, out=xa)
    ya = fused.rms_norm(xa, nw, 1e-5)
    xb = x0.clone()
    pend = dgemm.linear(a, wref, defer=True)
    yb = fused.rms_norm(xb, nw, 1e-5, pending=pend)
    assert torch.equal(xa.cpu(), xb.cpu()) and torch.equal(ya.cpu(), yb.cpu())
    pend = dgemm.linear(a, wref, defer=True)
    dgemm.linear(a, wref)
    with pytest.raises(RuntimeError):
        fused.rms_norm(x0.clone(), nw, 1e-5, pending=pend)
    # qkv: store epilogue in rope_kv
    B, hq, hkv, hd, T, pos = m, 12, 2, 64, 24, 5
    n = (hq + 2 * hkv) * hd
    wq = (torch.randn(n, k, generator=g) * 0.02).to(torch.bfloat16)
    qbuf = dgemm.frag_permute(wq).contiguous().to(dv)
    qref = dgemm.WeightRef(qbuf.data_ptr(), 0, n, k, dgemm.MODE_RAW)
    cos, sin = D.rope_tables(hd, T, 500000.0, "cpu")
    ca = torch.zeros(2, B, hkv, T, hd, dtype=torch.bfloat16, device=dv)
    cb = ca.clone()
    qa = fused.rope_kv(dgemm.linear(a, qref), cos[pos].to(dv), sin[pos].to(dv), ca, pos, hq, hkv)
    qb = fused.rope_kv(dgemm.linear(a, qref, defer=True), cos[pos].to(dv), sin[pos].to(dv), cb, pos, hq, hkv)
    assert torch.equal(qa.cpu(), qb.cpu()) and torch.equal(ca.cpu(), cb.cpu())


def _check_fragment_ordered_activations(gpu):
    """Producers writing the decode GEMM's fragment-ordered activations
    (RMSNorm, attention, the SiLU-mul epilogue) match the row-major results
    permuted by dgemm.to_frag, and the GEMM reading them gives the row-major
    GEMM's bits - raw (the pipelined kernels), BF11-packed (k_dgemm) - for row
    counts that are not a multiple of 16."""
    from ogkm.ops import bf12, dgemm
    dv = _dev(gpu)
    g = torch.Generator().manual_seed(21)
    m, d = 7, 1024
    x = (torch.randn(m, d, generator=g) * 2).to(torch.bfloat16).to(dv)
    nw = (torch.rand(d, generator=g) + 0.5).to(torch.bfloat16).to(dv)
    y = fused.rms_norm(x, nw, 1e-5)
    yf = fused.rms_norm(x, nw, 1e-5, out_frag=True)
    assert yf.shape == (16, d)
    assert torch.equal(dgemm.from_frag(yf, m).cpu(), y.cpu())
    B, hq, hkv, hd, T = m, 8, 2, 64, 300
    q = torch.randn(B, hq, hd, generator=g).to(torch.bfloat16).to(dv)
    cache = torch.randn(2, B, hkv, T, hd, generator=g).to(torch.bfloat16).to(dv)
    att = fused.attention(q, cache, 290)
    attf = fused.attention(q, cache, 290, out_frag=True)
    assert torch.equal(dgemm.from_frag(attf, B).cpu(), att.cpu())
    for packed in (False, True):
        n, k = 320, d
        wt = (torch.randn(n, k, generator=g) * 0.02).to(torch.bfloat16)
        flat = dgemm.frag_permute(wt).contiguous()
        if packed:
            stream, _ = bf12.pack(flat, chunk_values=1 << 16, fmt="bf11s")
            buf = stream.to(dv)
            ref = dgemm.WeightRef(buf.data_ptr(), 0, n, k, dgemm.packed_mode(stream), 16)
        else:
            buf = flat.to(dv)
            ref = dgemm.WeightRef(buf.data_ptr(), 0, n, k, dgemm.MODE_RAW)
        o_row = dgemm.linear(y, ref)
        o_frag = dgemm.linear(yf, ref, x_rows=m)
        assert torch.equal(o_row.cpu(), o_frag.cpu())
        # SiLU-mul epilogue into two column ranges of a fragment-ordered buffer
        gf = torch.zeros(16, 2 * (n // 2), dtype=torch.bfloat16, device=dv)
        s_row = dgemm.linear(y, ref, "silu_mul")
        dgemm.linear(yf, ref, "silu_mul", out=gf, out_frag=True, out_col0=0, x_rows=m)
        dgemm.linear(yf, ref, "silu_mul", out=gf, out_frag=True, out_col0=n // 2, x_rows=m)
        both = dgemm.from_frag(gf, m)
        assert torch.equal(both[:, :n // 2].cpu(), s_row.cpu()) and torch.equal(both[:, n // 2:].cpu(), s_row.cpu())


def test_fragment_ordered_activations_cpu(fake_rt):
    _check_fragment_ordered_activations(False)


@pytest.mark.gpu
def test_fragment_ordered_activations_gpu(gpu_rt):
    _check_fragment_ordered_activations(True)


def test_deferred_epilogues_cpu(fake_rt):
    _check_deferred_epilogues(False)


@pytest.mark.gpu
@pytest.mark.parametrize("d", [1024, 4096, 8192])
def test_deferred_epilogues_gpu(gpu_rt, d):
    _check_deferred_epilogues(True, d)


def test_rmsnorm_cpu(fake_rt):
    _check_rmsnorm(False)


def test_rope_kv_cpu(fake_rt):
    _check_rope_kv(False)


@pytest.mark.parametrize("length", [1, 255, 256, 257, 700])
def test_attention_cpu(fake_rt, length):
    _check_attention(False, length)


@pytest.mark.gpu
@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("dim", [512, 1024, 2048, 4096, 5120, 8192, 16384])
def test_rmsnorm_gpu(gpu_rt, dim, wide, monkeypatch):
    """One workgroup per row (dim <= 1024) and the multi-workgroup form (one per
    1024 columns, the row's last arriver normalises), ragged last quarter (5120);
    wide: the two-launch form (k_norm_ssq + k_norm_scale, OGKM_WIDE_NORM=1)."""
    monkeypatch.setattr(fused, "WIDE_NORM", wide)
    _check_rmsnorm(True, dim)


@pytest.mark.gpu
def test_rope_kv_gpu(gpu_rt):
    _check_rope_kv(True)


@pytest.mark.gpu
@pytest.mark.parametrize("length", [1, 255, 256, 257, 700])
def test_attention_gpu(gpu_rt, length):
    _check_attention(True, length)


# The GQA group shapes every tp8 rank of Llama-3 70B (8 q heads : 1 kv head) and
# 405B (16 : 1) runs.
@pytest.mark.parametrize("hq,hkv", [(8, 1), (16, 1)])
@pytest.mark.parametrize("length", [1, 700])
def test_attention_one_kv_head_cpu(fake_rt, hq, hkv, length):
    _check_attention(False, length, hq, hkv)


@pytest.mark.gpu
@pytest.mark.parametrize("hq,hkv", [(8, 1), (16, 1)])
@pytest.mark.parametrize("length", [1, 255, 256, 257, 700])
def test_attention_one_kv_head_gpu(gpu_rt, hq, hkv, length):
    _check_attention(True, length, hq, hkv)


@pytest.mark.gpu
@pytest.mark.parametrize("hq,hkv,hd", [(32, 8, 128), (16, 4, 64), (8, 1, 64), (4, 4, 128), (12, 2, 128), (16, 1, 128)])
@pytest.mark.parametrize("length", [1, 63, 64, 65, 700])
@pytest.mark.parametrize("split_tokens", [64, 256])
def test_attention_group_shapes_gpu(gpu_rt, hq, hkv, hd, length, split_tokens):
    """Every group-size / head-dim instantiation of the wave-split kernel
    (group 1..16 rounded up to 4 / 8 / 16, hd 64 / 128), partial waves included,
    in both workgroup shapes: 256-token four-wave splits and 64-token one-wave
    splits (an explicit option; measured slower at the bench shapes, profiles/r3_attn_split.txt)."""
    _check_attention(True, length, hq, hkv, hd, split_tokens)


# KV-read rate guards at ~85 % of the measured MALL-cold rates (tools/bench_attn.py,
# profiles/r4_attn_variants.txt: 8B 4.28, 70B 3.69, 70B-tp8 1.42 TB/s).
@pytest.mark.gpu
@pytest.mark.parametrize("name,B,hq,hkv,floor_tbps", [("8b", 64, 32, 8, 3.6), ("70b", 64, 64, 8, 3.1),
                                                      ("70b-tp8", 64, 8, 1, 1.2)])
def test_attention_gpu_kv_rate(gpu_rt, name, B, hq, hkv, floor_tbps):
    hd, L = 128, 1025
    q = torch.randn(B, hq, hd, device="cuda").to(torch.bfloat16)
    kvb = 2 * B * hkv * L * hd * 2
    ncopy = max(1, -(-(1 << 30) // kvb))  # rotate over >= 1 GB: past the 256 MB MALL
    caches = [torch.randn(2, B, hkv, L, hd, device="cuda").to(torch.bfloat16) for _ in range(ncopy)]
    for i in range(3):
        fused.attention(q, caches[i % ncopy], L)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 30
    e0.record()
    for i in range(iters):
        fused.attention(q, caches[i % ncopy], L)
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) / 1e3 / iters
    tbps = kvb / sec / 1e12
    print(f"attention {name}: {sec * 1e6:.1f} us, {tbps:.2f} TB/s of KV")
    assert tbps > floor_tbps
