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


def _check_rmsnorm(gpu):
    x = (torch.randn(5, 1024) * 3).to(torch.bfloat16)
    w = (torch.rand(1024) + 0.5).to(torch.bfloat16)
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


def _check_attention(gpu, length, hq=16, hkv=2, hd=128):
    B, T = 2, 700
    q = torch.randn(B, hq, hd).to(torch.bfloat16)
    cache = torch.randn(2, B, hkv, T, hd).to(torch.bfloat16)
    want = D.gqa_decode_attention(q.float(), cache[0].float(), cache[1].float(), length)
    dv = _dev(gpu)
    got = fused.attention(q.to(dv), cache.to(dv), length)
    torch.testing.assert_close(got.float().cpu(), want, atol=2e-2, rtol=2e-2)


def test_rmsnorm_cpu(fake_rt):
    _check_rmsnorm(False)


def test_rope_kv_cpu(fake_rt):
    _check_rope_kv(False)


@pytest.mark.parametrize("length", [1, 255, 256, 257, 700])
def test_attention_cpu(fake_rt, length):
    _check_attention(False, length)


@pytest.mark.gpu
def test_rmsnorm_gpu(gpu_rt):
    _check_rmsnorm(True)


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
@pytest.mark.parametrize("hq,hkv,hd", [(32, 8, 128), (16, 4, 64), (8, 1, 64), (4, 4, 128), (12, 2, 128)])
@pytest.mark.parametrize("length", [1, 63, 65, 700])
def test_attention_group_shapes_gpu(gpu_rt, hq, hkv, hd, length):
    """Every group-size / head-dim instantiation of the wave-split kernel
    (group 1..16 rounded up to 4 / 8 / 16, hd 64 / 128), partial waves included."""
    _check_attention(True, length, hq, hkv, hd)
