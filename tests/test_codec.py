"""Lossless weight codecs (csrc/core/codec.cpp): BF12 and BF11 blocks and the
self-describing streams built from them must round-trip every bf16 bit pattern.
CPU only; the GPU decoders are checked bit-for-bit against these encoders in
tests/test_gpu_runtime.py."""
from __future__ import annotations

import pytest
import torch
from hypothesis import given, settings, strategies as st

from ogkm.ops import bf12


def _roundtrip(ref: torch.Tensor, fmt: str, chunk: int = bf12.CHUNK_VALUES):
    stream, info = bf12.pack(ref, chunk_values=chunk, fmt=fmt)
    out = bf12.unpack_host(stream, info)
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    return info


@pytest.mark.parametrize("std", [0.02, 1.0, 1e-3, 300.0])
def test_bf11_ratio_and_exactness_gaussian(std):
    torch.manual_seed(1)
    ref = (torch.randn((2 << 20) + 8) * std).to(torch.bfloat16)
    i11 = _roundtrip(ref, "bf11")
    i12 = _roundtrip(ref, "bf12")
    assert i11.ratio < 0.70 < 0.75 < i12.ratio < 0.76


def test_specials_and_exceptions_every_tile():
    torch.manual_seed(2)
    ref = (torch.randn(1 << 20) * 0.02).to(torch.bfloat16)
    specials = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 3.0e38, 1e-40, -2.5, 1.0],
                            dtype=torch.bfloat16)
    for t in range(32):  # one burst of out-of-code-space exponents in every 32768-value tile
        ref[t * 32768 + 100:t * 32768 + 109] = specials
    _roundtrip(ref, "bf11")


def test_incompressible_falls_back():
    ref = torch.randint(-32768, 32767, (1 << 20,), dtype=torch.int16).view(torch.bfloat16)
    info = _roundtrip(ref, "bf11")
    assert info.ratio <= 1.001


@settings(max_examples=40, deadline=None)
@given(n=st.integers(1, 40000).map(lambda k: 2 * k), std=st.sampled_from([0.02, 1.0, 1e-30, 1e30]),
       chunk=st.sampled_from([8192, 16384, 1 << 20]), seed=st.integers(0, 2**31 - 1))
def test_bf11_property_roundtrip(n, std, chunk, seed):
    g = torch.Generator().manual_seed(seed)
    ref = (torch.randn(n, generator=g) * std).to(torch.bfloat16)
    _roundtrip(ref, "bf11", chunk)


@pytest.mark.parametrize("std", [0.02, 1.0, 1e-3])
def test_ans_ratio_and_exactness_gaussian(std):
    """ANS1 (rANS-coded exponents) round-trips and beats BF11 by its entropy margin."""
    torch.manual_seed(1)
    ref = (torch.randn(3 << 20) * std).to(torch.bfloat16)
    ia = _roundtrip(ref, "ans")
    i11 = _roundtrip(ref, "bf11")
    assert ia.ratio < 0.675 and ia.ratio < i11.ratio - 0.02, (ia.ratio, i11.ratio)
    assert bf12.chunk_kinds(bf12.pack(ref, fmt="ans")[0]) == {3}


def test_ans_specials_constant_incompressible_and_tails():
    torch.manual_seed(3)
    ref = (torch.randn(1 << 20) * 0.02).to(torch.bfloat16)
    specials = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 3.0e38, 1e-40, -2.5, 1.0],
                            dtype=torch.bfloat16)
    for t in range(32):  # rare exponents in every segment (12-bit frequency floor)
        ref[t * 32768 + 100:t * 32768 + 109] = specials
    _roundtrip(ref, "ans")
    _roundtrip(torch.zeros(1 << 16, dtype=torch.bfloat16), "ans")          # one symbol
    _roundtrip(torch.full((1 << 16,), 0.5, dtype=torch.bfloat16), "ans")   # one symbol
    rnd = torch.randint(-32768, 32767, (1 << 20,), dtype=torch.int16).view(torch.bfloat16)
    assert _roundtrip(rnd, "ans").ratio <= 1.001                           # raw fallback
    tail = (torch.randn((1 << 20) + 1000) * 0.02).to(torch.bfloat16)       # last chunk not % 512: raw
    info = _roundtrip(tail, "ans")
    assert bf12.chunk_kinds(bf12.pack(tail, fmt="ans")[0]) == {0, 3} and info.ratio < 0.68


@settings(max_examples=30, deadline=None)
@given(n=st.integers(1, 80).map(lambda k: 512 * k), std=st.sampled_from([0.02, 1.0, 1e-30, 1e30]),
       chunk=st.sampled_from([8192, 32768, 1 << 20]), seed=st.integers(0, 2**31 - 1))
def test_ans_property_roundtrip(n, std, chunk, seed):
    g = torch.Generator().manual_seed(seed)
    ref = (torch.randn(n, generator=g) * std).to(torch.bfloat16)
    _roundtrip(ref, "ans", chunk)


def _strided_rows_case(dev: str, fmt: str):
    """Rows of 4 chunks (a KV row block longer than the largest chunk) unpacked
    into a strided cache: row r lands at r * stride, its chunks back to back."""
    from ogkm.ops import bf12

    cv, rows, stride = 8192, 3, 4 * 8192 + 1000
    src = (torch.randn(rows, 4 * cv) * 0.7).to(torch.bfloat16)
    st, info = bf12.pack(src.reshape(-1), chunk_values=cv, fmt=fmt)
    assert info.nchunks == rows * 4
    dst = torch.full((rows * stride,), -7.0, dtype=torch.bfloat16, device=dev)
    s = st.to(dev)
    bf12.unpack_into(dst, s.data_ptr(), info, 0, 0 if dev == "cpu" else None, dst_stride=stride, row_chunks=4)
    if dev != "cpu":
        torch.cuda.synchronize()
    got = dst.cpu().view(rows, stride)
    assert torch.equal(got[:, :4 * cv].view(torch.int16), src.view(torch.int16))
    assert bool((got[:, 4 * cv:] == -7.0).all())  # the tail room is untouched


@pytest.mark.parametrize("fmt", ["bf11", "ans"])
def test_unpack_rows_of_chunks_into_strided_cache_cpu(fake_rt, fmt):
    _strided_rows_case("cpu", fmt)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["bf11", "bf12", "ans"])
def test_unpack_rows_of_chunks_into_strided_cache_gpu(gpu_rt, fmt):
    _strided_rows_case("cuda", fmt)
