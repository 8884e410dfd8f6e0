"""Tiered Llama decode on a real MI355X: the HIP decode GEMM (raw / BF11 in
registers / BF12 staged), the BF11 KV cache and the streaming ring against the
plain fp32 PyTorch reference (llama.reference_step), and lossless formats
against each other bit for bit."""
from __future__ import annotations

import pytest
import torch

from ogkm import rt
from ogkm._native import lib
from ogkm.models import llama

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("weight_format,kv_format", [("bf11", "bf11"), ("bf16", "bf16"), ("bf12", "bf16"), ("ans", "ans")])
def test_tiny_decode_matches_fp32_reference_gpu(gpu_rt, weight_format, kv_format):
    cfg = llama.CONFIGS["tiny"]
    m = llama.TieredLlama(cfg, batch=3, context=128, max_new_tokens=4, oversub=1.5, lookahead=1, seed=5,
                          weight_format=weight_format, kv_format=kv_format)
    m.keep_logits = True
    tok = torch.tensor([3, 11, 500], device="cuda")
    for _ in range(3):
        ref = llama.reference_step(cfg, m, tok.cpu(), m.pos).cpu()
        tok = m.step(tok)
        torch.cuda.synchronize()
        torch.testing.assert_close(m.last_logits.cpu(), ref, atol=0.05, rtol=0.05)
        tok = ref.argmax(-1).cuda()
    s = lib.stats()
    assert s["bytes_xfer_htd"] > 0  # oversubscribed: something streamed
    m.close()


def test_formats_bit_identical_gpu(gpu_rt):
    """Lossless resting formats give bit-identical logits when the same GEMM
    kernel family reads them: raw bf16 and rANS (unpacked to bf16 first)
    through k_dgemm_pipe; BF11 (decoded in k_dgemm's registers) against raw
    bf16 on k_dgemm<RAW>. The two families differ only in f32 summation order."""
    from ogkm.ops import dgemm
    cfg = llama.CONFIGS["small"]
    outs = {}
    pipe0 = dgemm.PIPE
    try:
        for tag, wf, kf, pipe in (("bf16", "bf16", "bf16", 1), ("bf16-split", "bf16", "bf16", 0),
                                  ("bf11", "bf11", "bf11", 0), ("ans", "ans", "ans", 1)):
            dgemm.PIPE = pipe
            m = llama.TieredLlama(cfg, batch=4, context=128, max_new_tokens=4, oversub=2.0, lookahead=1, seed=7,
                                  weight_format=wf, kv_format=kf)
            m.keep_logits = True
            tok = torch.tensor([1, 2, 3, 4], device="cuda")
            logs = []
            for _ in range(3):
                tok = m.step(tok)
                logs.append(m.last_logits.clone())
            torch.cuda.synchronize()
            outs[tag] = logs
            m.close()
    finally:
        dgemm.PIPE = pipe0
    for a, b in zip(outs["bf16"], outs["ans"]):
        assert torch.equal(a, b)
    for a, b in zip(outs["bf16-split"], outs["bf11"]):
        assert torch.equal(a, b)
    # the first step's logits agree across kernel families (later steps may pick
    # different argmax tokens on near-ties)
    torch.testing.assert_close(outs["bf16"][0], outs["bf16-split"][0], atol=0.05, rtol=0.05)


@pytest.mark.parametrize("kv_format", ["bf16", "ans"])
def test_kv_tiering_matches_fp32_reference_and_resident_kv_gpu(gpu_rt, kv_format):
    """KV prefixes as streamed per-layer units on the GPU: logits match the fp32
    reference and are bit-identical to the resident-KV run."""
    cfg = llama.CONFIGS["small"]
    outs = {}
    for tier in (False, True):
        m = llama.TieredLlama(cfg, batch=4, context=128, max_new_tokens=4, oversub=2.0, lookahead=1, seed=13,
                              weight_format="ans", kv_format=kv_format, kv_tiering=tier)
        m.keep_logits = True
        tok = torch.tensor([5, 17, 900, 33], device="cuda")
        logs = []
        for _ in range(3):
            ref = llama.reference_step(cfg, m, tok.cpu(), m.pos).cpu() if tier else None
            tok = m.step(tok)
            torch.cuda.synchronize()
            logs.append(m.last_logits.cpu())
            if tier:
                torch.testing.assert_close(logs[-1], ref, atol=0.05, rtol=0.05)
        if tier:
            assert any(k[0] == "kv" for k in m.stream_seq)
        outs[tier] = logs
        m.close()
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)


def test_fused_epilogues_bit_identical_gpu(gpu_rt):
    """Deferred GEMM epilogues (k_rope_kv / k_rmsnorm sum the split-K partials)
    vs the separate k_dgemm_reduce launches: identical logits."""
    cfg = llama.CONFIGS["small"]
    outs = {}
    for fuse in ((False, False), (True, False), (False, True), (True, True)):  # (deferred epilogues, frag x)
        m = llama.TieredLlama(cfg, batch=4, context=128, max_new_tokens=4, oversub=2.0, lookahead=1, seed=7,
                              weight_format="bf16", kv_format="bf16")
        m.fuse_epilogues, m.x_frag = fuse
        m.keep_logits = True
        tok = torch.tensor([1, 2, 3, 4], device="cuda")
        logs = []
        for _ in range(3):
            tok = m.step(tok)
            logs.append(m.last_logits.clone())
        torch.cuda.synchronize()
        outs[fuse] = logs
        m.close()
    for key in list(outs)[1:]:
        for a, b in zip(outs[(False, False)], outs[key]):
            assert torch.equal(a, b)
