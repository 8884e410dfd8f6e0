"""Tiered Llama decode: numerics vs a plain fp32 PyTorch reference, streaming
accounting vs the residency plan, and tensor parallelism over 2 processes (gloo)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from ogkm import rt
from ogkm._native import lib
from ogkm.models import llama

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kv_format,context", [("bf16", 8), ("bf11", 128)])
def test_tiny_decode_matches_fp32_reference(fake_rt, kv_format, context):
    cfg = llama.CONFIGS["tiny"]
    m = llama.TieredLlama(cfg, batch=2, context=context, max_new_tokens=4, oversub=1.5, lookahead=1, seed=5,
                          kv_format=kv_format)
    m.keep_logits = True
    tok = torch.tensor([3, 11])
    for _ in range(3):
        ref = llama.reference_step(cfg, m, tok, m.pos)
        tok = m.step(tok)
        torch.testing.assert_close(m.last_logits, ref, atol=0.05, rtol=0.05)
        # greedy pick agrees with the fp32 reference up to bf16 near-ties
        picked = ref.gather(1, tok.view(-1, 1)).squeeze(1)
        assert bool((ref.max(-1).values - picked <= 0.05).all())
        tok = ref.argmax(-1)  # continue both paths from the reference tokens
    m.close()


def test_streaming_matches_plan_runtime_packed(fake_rt):
    """bf16 weights, BF12 host copies decoded inside the H2D copy (runtime-packed ranges)."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, lock_check=1, host_budget_mb=1024)
    cfg = llama.CONFIGS["small"]
    m = llama.TieredLlama(cfg, batch=2, context=8, max_new_tokens=8, oversub=2.0, lookahead=1, weight_format="bf16")
    assert 1.9 < m.footprint / m.budget < 2.1
    tok = torch.tensor([1, 2])
    tok = m.step(tok)
    tok = m.step(tok)
    lib.reset_counters()
    steps = 3
    for _ in range(steps):
        tok = m.step(tok)
    s = lib.stats()
    per_step = s["decoded_bytes"] / steps
    # every streamed tensor is delivered once per step (+/- the wrap-around prefetch)
    assert 0.9 * m.streamed_bytes <= per_step <= 1.15 * m.streamed_bytes, (per_step, m.streamed_bytes)
    # ... while only the BF12-packed bytes cross the link (lossless, ~0.75x)
    assert s["bytes_xfer_htd"] < 0.8 * s["decoded_bytes"]
    assert s["bytes_xfer_dth"] == 0  # streamed weights are clean read-duplicates: never written back
    m.close()


@pytest.mark.parametrize("fmt,ratio", [("bf12", 0.8), ("bf11", 0.74)])
def test_streaming_matches_plan_hbm_packed(fake_rt, fmt, ratio):
    """bf11/bf12 weights: packed in every tier, unpacked into the staging buffer per layer."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, lock_check=1, host_budget_mb=1024)
    cfg = llama.CONFIGS["small"]
    m = llama.TieredLlama(cfg, batch=2, context=8, max_new_tokens=8, oversub=2.0, lookahead=1, weight_format=fmt)
    assert 1.9 < m.footprint / m.budget < 2.1
    assert m.res_layer_bytes < ratio * m.layer_bytes
    tok = torch.tensor([1, 2])
    tok = m.step(tok)
    tok = m.step(tok)
    lib.reset_counters()
    steps = 3
    for _ in range(steps):
        tok = m.step(tok)
    s = lib.stats()
    per_step = s["bytes_xfer_htd"] / steps
    assert 0.9 * m.streamed_bytes <= per_step <= 1.15 * m.streamed_bytes, (per_step, m.streamed_bytes)
    assert s["bytes_xfer_dth"] == 0
    # more layers fit than with raw weights under the same budget
    assert sum(m.resident) >= 1
    m.close()


def test_bf12_weights_bit_identical_to_bf16(fake_rt):
    cfg = llama.CONFIGS["tiny"]
    out = {}
    for fmt in ("bf16", "bf12", "bf11", "ans"):
        m = llama.TieredLlama(cfg, batch=2, context=8, max_new_tokens=4, oversub=1.5, lookahead=1, seed=9,
                              weight_format=fmt)
        m.keep_logits = True
        tok = torch.tensor([5, 7])
        logs = []
        for s in range(3):
            m.step(tok + s)
            logs.append(m.last_logits.clone())
        out[fmt] = logs
        m.close()
    for fmt in ("bf12", "bf11", "ans"):
        for a, b in zip(out["bf16"], out[fmt]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("fmt", ["bf16", "ans"])
def test_fused_epilogues_bit_identical_to_separate_reduces(fake_rt, fmt):
    """Deferred GEMM epilogues (qkv sum in rope_kv, o / down residual adds in
    the next RMSNorm) give the same logits bit for bit as the separate
    k_dgemm_reduce launches, streamed (oversubscribed) and resident."""
    cfg = llama.CONFIGS["tiny"]
    out = {}
    for fuse in ((False, False), (True, False), (False, True), (True, True)):  # (deferred epilogues, frag x)
        m = llama.TieredLlama(cfg, batch=3, context=8, max_new_tokens=4, oversub=1.5, lookahead=1, seed=4,
                              weight_format=fmt)
        m.fuse_epilogues, m.x_frag = fuse
        m.keep_logits = True
        logs = []
        tok = torch.tensor([5, 7, 9])
        for _ in range(3):
            tok = m.step(tok)
            logs.append(m.last_logits.clone())
        out[fuse] = logs
        m.close()
    for key in list(out)[1:]:
        for a, b in zip(out[(False, False)], out[key]):
            assert torch.equal(a, b)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _single_run(batch: int = 2, oversub: float = 1.2, model: str = "tiny"):
    cfg = llama.CONFIGS[model]
    m = llama.TieredLlama(cfg, batch=batch, context=8, max_new_tokens=4, oversub=oversub, lookahead=1, seed=5)
    m.keep_logits = True
    single = []
    for s in range(3):
        tok = m.step(torch.tensor([3 + s + 8 * j for j in range(batch)]))
        single.append((tok.tolist(), m.last_logits[:, :64].clone()))
    m.close()
    return single


def _multi_run(nproc: int, parallel: str, batch: int = 2, oversub: float = 1.2, model: str = "tiny"):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", PARALLEL=parallel, BATCH=str(batch),
               OVERSUB=str(oversub), MODEL=model)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests/helpers/tp_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    line = [l for l in r.stdout.splitlines() if l.startswith("TPRESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(line[0][len("TPRESULT "):])


def test_tensor_parallel_two_ranks_matches_single(fake_rt):
    single = _single_run()
    tp = _multi_run(2, "tp")
    assert len(tp) == 4
    for (tok1, log1), step in zip(single, tp):
        torch.testing.assert_close(torch.tensor(step["logits"]), log1, atol=0.05, rtol=0.05)


def test_peer_shards_two_ranks_matches_single(fake_rt):
    """Config 4 ("peermem-style P2P shards"): each rank owns half of every unit,
    units are all-gathered before use and each rank decodes its own sequences
    with the full model - the same math as one GPU, at 2x oversubscription of the
    per-rank shard footprint."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, lock_check=1, host_budget_mb=2048)
    single = _single_run(batch=4, oversub=2.0, model="small")
    sh = _multi_run(2, "shards", batch=4, oversub=2.0, model="small")
    assert len(sh) == 4 and sh[-1]["gathers"] > 0
    for (tok1, log1), step in zip(single, sh):
        torch.testing.assert_close(torch.tensor(step["logits"]), log1, atol=1e-3, rtol=1e-3)
        assert step["tokens"] == tok1[:2]  # rank 0's own sequences


def test_peer_shards_keep_read_duplicates_when_hbm_allows(fake_rt):
    """Shards mode with HBM to spare (no oversubscription): whole gathered units
    stay as read duplicates in a managed buffer the runtime accounts for - the
    first step all-gathers every unit once, later steps gather nothing - and
    the logits still match one GPU."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, lock_check=1, host_budget_mb=2048)
    single = _single_run(batch=4, oversub=1.0, model="small")
    # budget 2.5x the rank's shard footprint: room for every whole unit
    sh = _multi_run(2, "shards", batch=4, oversub=0.4, model="small")
    assert len(sh) == 4 and sh[-1]["cache_bytes"] > 0 and sh[-1]["cache_hits"] > 0
    assert sh[1]["gathers"] == sh[0]["gathers"] == sh[2]["gathers"] > 0  # nothing gathered after step 1
    # budget 1x: part of the units duplicated, evenly over the use order
    part = _multi_run(2, "shards", batch=4, oversub=1.0, model="small")
    per_step = part[2]["gathers"] - part[1]["gathers"]
    assert part[-1]["cache_bytes"] > 0 and 0 < per_step < part[0]["gathers"]
    for (tok1, log1), step in zip(single, part):
        torch.testing.assert_close(torch.tensor(step["logits"]), log1, atol=1e-3, rtol=1e-3)
    for (tok1, log1), step in zip(single, sh):
        torch.testing.assert_close(torch.tensor(step["logits"]), log1, atol=1e-3, rtol=1e-3)
        assert step["tokens"] == tok1[:2]


def test_three_tier_host_and_cxl_streaming(fake_rt):
    """Config 5 shape: HBM + host DRAM + CXL.mem. Streamed tensors rest
    interleaved on the host and (emulated) CXL tiers; decode output is identical
    to the two-tier run and every step streams the planned bytes."""
    from ogkm import cxl

    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, lock_check=1, host_budget_mb=1024)
    cxl.rediscover(lib.host_node(), "/sys")
    cfg = llama.CONFIGS["small"]
    outs = {}
    for tiers in ("host", "host+cxl"):
        m = llama.TieredLlama(cfg, batch=2, context=8, max_new_tokens=8, oversub=2.0, lookahead=1, seed=3,
                              tiers=tiers)
        m.keep_logits = True
        tok = torch.tensor([4, 9])
        logs = []
        for s in range(3):
            m.step(tok + s)
            logs.append(m.last_logits.clone())
        outs[tiers] = logs
        if tiers == "host+cxl":
            assert m.cxl_streamed_bytes > 0
            locs = set()
            for key, b in m.ubuf.items():
                if not m._is_resident(key):
                    info = b.residency(0)
                    locs |= {x["tier"] for x in info["resident_on"]}
            assert {"cxl", "host"} <= locs, locs
        m.close()
    for a, b in zip(outs["host"], outs["host+cxl"]):
        assert torch.equal(a, b)


def test_bf11_kv_cache_bit_identical_to_bf16(fake_rt):
    """The packed (BF11 prefix + raw tail) KV cache decodes the exact bf16
    context: logits are bit-identical to the raw cache, and it rests smaller."""
    cfg = llama.CONFIGS["tiny"]
    out, res = {}, {}
    for fmt in ("bf16", "bf11", "ans"):
        m = llama.TieredLlama(cfg, batch=2, context=128, max_new_tokens=4, oversub=1.2, lookahead=1, seed=9,
                              kv_format=fmt)
        m.keep_logits = True
        tok = torch.tensor([5, 7])
        logs = []
        for s in range(3):
            tok = m.step(tok)
            logs.append(m.last_logits.clone())
        out[fmt] = logs
        res[fmt] = m.kv_resident_bytes
        m.close()
    for fmt in ("bf11", "ans"):
        for a, b in zip(out["bf16"], out[fmt]):
            assert torch.equal(a, b)
    assert res["ans"] < res["bf11"] < 0.8 * res["bf16"]


def test_planner_off_matches_static_plan(fake_rt):
    """planner='off': no resident plan, no lifetime pins - every unit prefers
    HBM and the runtime's LRU evicts under 2x oversubscription. Logits equal the
    planned run's, and the runtime (not the plan) did the evicting."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, lock_check=1, host_budget_mb=1024)
    cfg = llama.CONFIGS["small"]
    out = {}
    for planner in ("static", "off"):
        m = llama.TieredLlama(cfg, batch=2, context=8, max_new_tokens=4, oversub=2.0, lookahead=1, seed=3,
                              weight_format="ans", planner=planner)
        m.keep_logits = True
        if planner == "off":
            assert m.describe()["resident_layers"] == 0 and not m._pin_leases
        lib.reset_counters()
        logs = []
        for s in range(3):
            m.step(torch.tensor([5, 7]) + s)
            logs.append(m.last_logits.clone())
        out[planner] = (logs, lib.stats()["evictions"])
        if planner == "off":
            assert not m._pin_leases   # nothing pinned for the model's lifetime
        m.close()
    for a, b in zip(out["static"][0], out["off"][0]):
        assert torch.equal(a, b)
    assert out["off"][1] > 0


@pytest.mark.parametrize("kv_format", ["bf16", "ans"])
def test_kv_tiering_bit_identical_to_resident_kv(fake_rt, kv_format):
    """KV tiering: each layer's prefilled KV is a managed unit that streams with
    its layer (evicted past the budget, prefetched ahead); logits are
    bit-identical to the resident-KV run and KV units really were streamed."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, lock_check=1, host_budget_mb=1024)
    cfg = llama.CONFIGS["tiny"]
    out = {}
    for tier in (False, True):
        m = llama.TieredLlama(cfg, batch=2, context=128, max_new_tokens=4, oversub=2.0, lookahead=1, seed=11,
                              kv_format=kv_format, weight_format="bf16", kv_tiering=tier)
        m.keep_logits = True
        logs = []
        for s in range(3):
            m.step(torch.tensor([3, 9]) + s)
            logs.append(m.last_logits.clone())
        if tier:
            streamed_kv = [k for k in m.stream_seq if k[0] == "kv"]
            assert streamed_kv, "some KV prefixes must stream at 2x oversubscription"
            assert m.describe()["kv_tiering"]
            for i in range(cfg.n_layers):   # the host view of the tiered cache matches the resident one
                assert torch.equal(m.host_kv(i), out[False][1][i])
        out[tier] = (logs, [m.host_kv(i) for i in range(cfg.n_layers)])
        m.close()
    for a, b in zip(out[False][0], out[True][0]):
        assert torch.equal(a, b)


def test_long_context_packed_kv_rows_of_chunks(fake_rt):
    """A context whose (k|v, b, head) row block exceeds the largest codec chunk
    (ctx * hd = 2 Mi values = 2 chunks) still rests packed and decodes the exact
    bf16 context (the unpack lands each row's chunks back to back in the cache)."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, host_budget_mb=2048)
    cfg = llama.CONFIGS["tiny"]
    ctx = (2 << 20) // cfg.head_dim
    out = {}
    for fmt in ("bf16", "ans"):
        m = llama.TieredLlama(cfg, batch=1, context=ctx, max_new_tokens=3, oversub=1.0, lookahead=1, seed=4,
                              kv_format=fmt, weight_format="bf16")
        assert fmt == "bf16" or m.kv_row_chunks == 2
        m.keep_logits = True
        m.step(torch.tensor([3]))
        out[fmt] = m.last_logits.clone()
        m.close()
    assert torch.equal(out["bf16"], out["ans"])


def test_planner_off_next_use_streams_like_the_plan(fake_rt, monkeypatch):
    """planner='off' with next-use hints (each streamed unit is next used one
    pass later) and nothing else from the model: the arena evicts in Belady
    order, keeping a fixed subset resident as the static plan does by hand -
    the bytes streamed per step come within 10% of the plan's, and below the
    hint-less (recency) run's. With the runtime's spread classes (the default,
    perf_spread_enable: it splits the hinted units into a keep class sized to
    its arena, spread over the use order, and a stream class evicted first) the
    order is no longer pure Belady: it stays below the recency run and within
    25% of the plan on this small model, whose prefetch window is a large share
    of the arena - and the runtime, not the model, found the classes."""
    lib.shutdown()
    rt.init("fake", fake_devices=1, fake_hbm_mb=1024, host_budget_mb=4096)
    cfg = llama.CONFIGS["small"]
    htd, spread_st = {}, {}
    for name, planner, nu, spread in (("static", "static", "1", 1), ("lru", "off", "0", 1),
                                      ("next_use", "off", "1", 0), ("spread", "off", "1", 1)):
        monkeypatch.setenv("OGKM_NEXT_USE", nu)
        lib.configure("perf_spread_enable", spread)
        m = llama.TieredLlama(cfg, batch=8, context=32, max_new_tokens=12, oversub=2.0, device=0, seed=1,
                              weight_format="ans", kv_format="bf16", planner=planner)
        assert m.next_use == (name in ("next_use", "spread"))
        tok = torch.arange(8) * 7
        for _ in range(3):
            tok = m.step(tok)
        lib.sync_all()
        lib.reset_counters()
        for _ in range(4):
            tok = m.step(tok)
        lib.sync_all()
        htd[name] = lib.stats()["bytes_xfer_htd"] / 4
        spread_st[name] = lib.spread_stats(0)
        m.close()
    lib.configure("perf_spread_enable", 1)
    assert htd["next_use"] < htd["lru"], htd
    assert htd["next_use"] <= 1.10 * htd["static"], htd
    # spread classes trade bytes for a link that streams throughout the step
    # (on the GPU: 129.4 vs 103 tok/s for plain Belady at 27.5 vs 27.6 GB/step,
    # profiles/r5_spread.md); on this tiny fake arena, whose contiguous
    # extents cut into kept chunks, they stream up to ~40 % over the plan
    assert htd["spread"] <= 1.45 * htd["static"], htd
    s = spread_st["spread"]
    assert s["ready"] and s["ranges"] > 0 and 0 < s["keep_ranges"] < s["ranges"], s
    assert spread_st["next_use"]["ranges"] == 0
