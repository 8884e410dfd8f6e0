"""Llama-3 decode with tiered (oversubscribed) weights on the ogkm runtime.

Every weight and the KV cache live in runtime-managed memory. The HBM arena is
capped at ``footprint / oversub`` (2x oversubscription = half the managed
footprint fits in HBM). A residency planner decides, per 2 MB-block range:

  * KV cache            preferred gpu, leased for the whole run (hot, written every step)
  * resident layers     preferred gpu (evicted last - the arena's preferred LRU list)
  * streamed layers     preferred host + read-mostly: each step the GPU gets a
                        read-duplicate copy through the migration ring (HIP copy
                        kernel on a side stream, layer-ahead prefetch), the clean
                        copy is dropped when the arena needs the space
  * token embedding     preferred host + accessed_by gpu: never migrated, rows are
                        gathered remotely by the residency-checking HIP kernel

The compute stream never blocks the host: it waits on ring fences GPU-side,
and the ring waits on the compute stream's release events before overwriting a
chunk (SURVEY.md §7.3 minimum slice: malloc_managed + residency map + HBM budget
+ evict to host + software faults + decode tokens/s).

Tensor parallelism (``tp_world`` > 1, one process per GPU, RCCL) shards every
layer Megatron-style; each rank streams only its shard over its own PCIe link.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import rt
from .._native import lib
from ..ops import decode as D
from ..ops.memory import managed_embedding
from ..parallel import comm, tp as tpmod

ALIGN = 4096


@dataclass(frozen=True)
class LlamaConfig:
    name: str
    dim: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn_dim: int
    vocab: int
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def params(self) -> int:
        hd = self.head_dim
        per_layer = (self.dim * (self.n_heads + 2 * self.n_kv_heads) * hd + self.n_heads * hd * self.dim
                     + 3 * self.dim * self.ffn_dim + 2 * self.dim)
        return self.n_layers * per_layer + 2 * self.vocab * self.dim + self.dim


CONFIGS = {
    "llama3-8b": LlamaConfig("llama3-8b", 4096, 32, 32, 8, 14336, 128256),
    "llama3-70b": LlamaConfig("llama3-70b", 8192, 80, 64, 8, 28672, 128256),
    "llama3-405b": LlamaConfig("llama3-405b", 16384, 126, 128, 8, 53248, 128256),
    "tiny": LlamaConfig("tiny", 512, 4, 8, 2, 1536, 4096),
    "small": LlamaConfig("small", 1024, 8, 16, 4, 2816, 8192),
}


def _al(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class LayerLayout:
    """Byte offsets of one TP shard's tensors inside a layer buffer (bf16, 4 KB aligned)."""

    shapes: dict = field(default_factory=dict)
    offsets: dict = field(default_factory=dict)
    nbytes: int = 0

    @staticmethod
    def build(cfg: LlamaConfig, world: int) -> "LayerLayout":
        hd = cfg.head_dim
        hq, hkv, f = cfg.n_heads // world, cfg.n_kv_heads // world, cfg.ffn_dim // world
        L = LayerLayout()
        for name, shape in (("attn_norm", (cfg.dim,)), ("wqkv", ((hq + 2 * hkv) * hd, cfg.dim)),
                            ("wo", (cfg.dim, hq * hd)), ("mlp_norm", (cfg.dim,)), ("wgu", (2 * f, cfg.dim)),
                            ("wd", (cfg.dim, f))):
            L.shapes[name] = shape
            L.offsets[name] = L.nbytes
            L.nbytes += _al(math.prod(shape) * 2)
        return L


class TieredLlama:
    def __init__(self, cfg: LlamaConfig, batch: int, context: int, max_new_tokens: int = 64, oversub: float = 2.0,
                 device: int = 0, tp_rank: int = 0, tp_world: int = 1, seed: int = 0, lookahead: int = 2,
                 hbm_budget: Optional[int] = None, init_std: float = 0.02, verbose: bool = False,
                 packed: bool = True):
        assert cfg.n_heads % tp_world == 0 and cfg.n_kv_heads % tp_world == 0 and cfg.ffn_dim % tp_world == 0
        assert cfg.vocab % tp_world == 0
        self.cfg, self.B, self.ctx = cfg, batch, context
        self.T = context + max_new_tokens
        self.dev = device
        self.rank, self.world = tp_rank, tp_world
        self.fake = lib.backend_name() == "fake"
        self.tdev = torch.device("cpu") if self.fake else torch.device("cuda", device)
        self.verbose = verbose
        self.layout = LayerLayout.build(cfg, tp_world)
        hd = cfg.head_dim
        self.hq, self.hkv = cfg.n_heads // tp_world, cfg.n_kv_heads // tp_world
        self.vocab_local = cfg.vocab // tp_world
        # ---- footprint and budget
        self.layer_bytes = self.layout.nbytes
        self.head_bytes = _al(self.vocab_local * cfg.dim * 2)
        self.embed_bytes = _al(cfg.vocab * cfg.dim * 2)
        self.kv_layer_bytes = 2 * batch * self.hkv * self.T * hd * 2
        self.kv_bytes = cfg.n_layers * self.kv_layer_bytes
        self.footprint = self.embed_bytes + cfg.n_layers * self.layer_bytes + self.head_bytes + self.kv_bytes
        self.oversub = oversub
        blk = 2 << 20
        budget = hbm_budget if hbm_budget is not None else int(self.footprint / oversub)
        self.budget = budget // blk * blk
        lib.init_device(device, self.budget)
        # ---- residency plan
        def chunks(n):
            return (n + blk - 1) // blk * blk
        staging = (lookahead + 1) * chunks(max(self.layer_bytes, self.head_bytes))
        avail = self.budget - chunks(self.kv_bytes) - staging
        if avail < 0:
            raise ValueError(f"HBM budget {self.budget/2**30:.1f} GiB too small for KV + staging "
                             f"({(chunks(self.kv_bytes) + staging)/2**30:.1f} GiB)")
        n_res = max(0, min(cfg.n_layers, avail // chunks(self.layer_bytes)))
        left = avail - n_res * chunks(self.layer_bytes)
        self.head_resident = left >= chunks(self.head_bytes)
        # spread resident layers evenly so streaming continues behind them
        self.resident = [((i + 1) * n_res) // cfg.n_layers > (i * n_res) // cfg.n_layers for i in range(cfg.n_layers)]
        self.lookahead = lookahead
        self.window_bytes = lookahead * chunks(max(self.layer_bytes, self.head_bytes))
        self.streamed_bytes = (sum(self.layer_bytes for r in self.resident if not r)
                               + (0 if self.head_resident else self.head_bytes))
        # ---- allocate + init
        t0 = time.perf_counter()
        gpu = rt.Loc.gpu(device)
        host = rt.Loc.host()
        self.embed = rt.malloc_managed(self.embed_bytes, "embed")
        self.embed.set_preferred_location(host)
        self.embed.set_accessed_by(device)
        self.kv = rt.malloc_managed(self.kv_bytes, "kv")
        self.kv.set_preferred_location(gpu)
        # Streamed tensors keep a BF12-packed (lossless) host copy: the H2D copy
        # kernel decodes it on the fly, so ~25% fewer bytes cross PCIe per step.
        self.packed = packed
        self.layers = []
        for i in range(cfg.n_layers):
            b = rt.malloc_managed(self.layer_bytes, f"layer{i}", packed_bf16=packed and not self.resident[i])
            if self.resident[i]:
                b.set_preferred_location(gpu)
            else:
                b.set_preferred_location(host)
                b.set_read_mostly(True)
            self.layers.append(b)
        self.head = rt.malloc_managed(self.head_bytes, "lm_head", packed_bf16=packed and not self.head_resident)
        if self.head_resident:
            self.head.set_preferred_location(gpu)
        else:
            self.head.set_preferred_location(host)
            self.head.set_read_mostly(True)
        self._init_weights(seed, init_std)
        self.final_norm = torch.ones(cfg.dim, dtype=torch.bfloat16, device=self.tdev)
        self.cos, self.sin = D.rope_tables(hd, self.T, cfg.rope_theta, self.tdev)
        # KV cache: leased for the model's lifetime (hot, written every step)
        self.kv_lease = self.kv.acquire(device, rt.WRITE)
        self.kv_lease.wait()
        kv = self.kv_lease.tensor((cfg.n_layers, 2, batch, self.hkv, self.T, hd), torch.bfloat16)
        # Synthetic prefilled context, generated at full head count and sliced to
        # this rank's KV heads so every TP degree decodes the same model state.
        g = torch.Generator(device=self.tdev).manual_seed(seed + 7919)
        h0 = self.rank * self.hkv
        for i in range(cfg.n_layers):
            full = torch.empty(2, batch, cfg.n_kv_heads, context, hd, dtype=torch.bfloat16, device=self.tdev)
            full.normal_(0.0, 1.0, generator=g)
            kv[i, :, :, :, :context].copy_(full[:, :, h0:h0 + self.hkv])
            del full
        self.kv_t = kv
        self.pos = context
        # ---- streaming schedule: use order within a step
        self.order = [("layer", i) for i in range(cfg.n_layers)] + [("head", 0)]
        self.stream_seq = [k for k in self.order if not self._is_resident(k)]
        self._pf_next = 0           # next index in stream_seq to prefetch (cyclic)
        self._inflight: list = []   # prefetched, not yet consumed
        self._views: dict = {}
        self.keep_logits = False   # tests: keep the full-vocab logits of the last step
        self.last_logits = None
        self.init_seconds = time.perf_counter() - t0
        if verbose:
            self.describe()

    # ------------------------------------------------------------------ setup
    def describe(self) -> dict:
        d = {
            "model": self.cfg.name, "tp": f"{self.rank}/{self.world}", "batch": self.B, "context": self.ctx,
            "footprint_gb": self.footprint / 1e9, "hbm_budget_gb": self.budget / 1e9,
            "oversubscription": self.footprint / self.budget, "kv_gb": self.kv_bytes / 1e9,
            "layer_gb": self.layer_bytes / 1e9, "resident_layers": sum(self.resident),
            "streamed_layers": self.cfg.n_layers - sum(self.resident), "head_resident": self.head_resident,
            "streamed_gb_per_step": self.streamed_bytes / 1e9, "init_s": getattr(self, "init_seconds", None),
            "packed_host_copies": getattr(self, "packed", False),
        }
        if self.verbose and self.rank == 0:
            print("[ogkm] plan:", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}, flush=True)
        return d

    def _is_resident(self, key) -> bool:
        kind, i = key
        return self.resident[i] if kind == "layer" else self.head_resident

    def _buf(self, key) -> "rt.ManagedBuffer":
        kind, i = key
        return self.layers[i] if kind == "layer" else self.head

    def _init_weights(self, seed: int, std: float) -> None:
        cfg, L = self.cfg, self.layout
        hd = cfg.head_dim
        dev = self.tdev
        scratch = torch.empty(self.layer_bytes, dtype=torch.uint8, device=dev)

        def put(name, t):
            off = L.offsets[name]
            n = t.numel() * 2
            scratch[off:off + n].copy_(t.reshape(-1).view(torch.uint8))

        for i in range(cfg.n_layers):
            g = torch.Generator(device=dev).manual_seed(seed * 1000003 + i)
            wq = torch.empty(cfg.n_heads * hd, cfg.dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
            wk = torch.empty(cfg.n_kv_heads * hd, cfg.dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
            wv = torch.empty(cfg.n_kv_heads * hd, cfg.dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
            put("wqkv", tpmod.shard_qkv(wq, wk, wv, self.rank, self.world))
            del wq, wk, wv
            wo = torch.empty(cfg.dim, cfg.n_heads * hd, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
            put("wo", tpmod.shard_cols(wo, self.rank, self.world))
            del wo
            wg = torch.empty(cfg.ffn_dim, cfg.dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
            wu = torch.empty(cfg.ffn_dim, cfg.dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
            put("wgu", tpmod.shard_gate_up(wg, wu, self.rank, self.world))
            del wg, wu
            wd = torch.empty(cfg.dim, cfg.ffn_dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
            put("wd", tpmod.shard_cols(wd, self.rank, self.world))
            del wd
            one = torch.ones(cfg.dim, dtype=torch.bfloat16, device=dev)
            put("attn_norm", one)
            put("mlp_norm", one)
            self.layers[i].write(scratch)
        del scratch
        g = torch.Generator(device=dev).manual_seed(seed * 1000003 + 999983)
        emb = torch.empty(cfg.vocab, cfg.dim, dtype=torch.bfloat16, device=dev).normal_(0, 1.0, generator=g)
        self.embed.write(emb)
        head = torch.empty(cfg.vocab, cfg.dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
        self.head.write(tpmod.shard_rows(head, self.rank, self.world).contiguous())
        del emb, head
        if not self.fake:
            torch.cuda.synchronize(self.dev)

    # ------------------------------------------------------------------ streaming
    def _prefetch_ahead(self) -> None:
        """Keep up to ``window_bytes`` of upcoming streamed tensors in flight on the ring."""
        if not self.stream_seq:
            return
        inflight = sum(self._buf(k).size for k in self._inflight)
        n = len(self.stream_seq)
        while len(self._inflight) < n:
            key = self.stream_seq[self._pf_next]
            nb = self._buf(key).size
            if self._inflight and inflight + nb > self.window_bytes:
                break
            self._buf(key).prefetch(rt.Loc.gpu(self.dev))
            self._inflight.append(key)
            inflight += nb
            self._pf_next = (self._pf_next + 1) % n

    def _use(self, key):
        if not self._is_resident(key):
            if self._inflight and self._inflight[0] == key:
                self._inflight.pop(0)
            self._prefetch_ahead()
        lease = self._buf(key).acquire(self.dev, rt.READ)
        lease.wait(0 if self.fake else None)
        return lease

    def _layer_views(self, lease) -> dict:
        v = self._views.get(lease.dptr)
        if v is None:
            v = {name: rt._tensor_from_ptr(lease.dptr + self.layout.offsets[name], shape, torch.bfloat16,
                                           "cpu" if self.fake else "cuda", self.dev)
                 for name, shape in self.layout.shapes.items()}
            if len(self._views) > 4 * len(self.order):
                self._views.clear()
            self._views[lease.dptr] = v
        return v

    # ------------------------------------------------------------------ decode
    @torch.no_grad()
    def step(self, tokens: torch.Tensor) -> torch.Tensor:
        """One decode step for all B sequences: tokens [B] -> next tokens [B] (greedy)."""
        cfg, B = self.cfg, self.B
        hd = cfg.head_dim
        pos = self.pos
        assert pos < self.T, "KV cache full"
        self._prefetch_ahead()
        x = managed_embedding(self.embed, tokens, cfg.dim, torch.bfloat16, self.dev)
        if self.fake:
            x = x.to(self.tdev)
        cos, sin = self.cos[pos], self.sin[pos]
        for i in range(cfg.n_layers):
            lease = self._use(("layer", i))
            w = self._layer_views(lease)
            h = D.rms_norm(x, w["attn_norm"], cfg.norm_eps)
            qkv = h @ w["wqkv"].t()
            q = qkv[:, :self.hq * hd].view(B, self.hq, hd)
            k = qkv[:, self.hq * hd:(self.hq + self.hkv) * hd].view(B, self.hkv, hd)
            v = qkv[:, (self.hq + self.hkv) * hd:].view(B, self.hkv, hd)
            q = D.apply_rope(q, cos, sin)
            k = D.apply_rope(k, cos, sin)
            kc, vc = self.kv_t[i, 0], self.kv_t[i, 1]
            kc[:, :, pos].copy_(k)
            vc[:, :, pos].copy_(v)
            a = D.gqa_decode_attention(q, kc, vc, pos + 1)
            o = a @ w["wo"].t()
            x = x + tpmod.row_parallel_reduce(o)
            h = D.rms_norm(x, w["mlp_norm"], cfg.norm_eps)
            gu = h @ w["wgu"].t()
            d = D.silu_mul(gu) @ w["wd"].t()
            x = x + tpmod.row_parallel_reduce(d)
            lease.release(0 if self.fake else None)
        x = D.rms_norm(x, self.final_norm, cfg.norm_eps)
        lease = self._use(("head", 0))
        head = rt._tensor_from_ptr(lease.dptr, (self.vocab_local, cfg.dim), torch.bfloat16,
                                   "cpu" if self.fake else "cuda", self.dev)
        logits = x @ head.t()
        if self.keep_logits:
            self.last_logits = comm.all_gather_cat(logits.float(), dim=-1)
        nxt = tpmod.vocab_parallel_argmax(logits, self.rank, self.world)
        lease.release(0 if self.fake else None)
        self.pos += 1
        return nxt

    def reset(self, position: Optional[int] = None) -> None:
        self.pos = self.ctx if position is None else position

    def close(self) -> None:
        self.kv_lease.release(0 if self.fake else None)
        lib.sync_all()
        for b in [self.embed, self.kv, self.head] + self.layers:
            b.free()


def reference_step(cfg: LlamaConfig, model: TieredLlama, tokens: torch.Tensor, pos: int) -> torch.Tensor:
    """Plain-PyTorch fp32 reference of one decode step built from the same
    weights (read back through the runtime), for numerics tests on tiny configs."""
    hd = cfg.head_dim
    dev = model.tdev
    B = tokens.shape[0]
    emb = model.embed.read().view(torch.bfloat16).view(cfg.vocab, cfg.dim).float()
    x = emb[tokens.cpu()].to(dev)
    cos, sin = model.cos[pos], model.sin[pos]
    for i in range(cfg.n_layers):
        raw = model.layers[i].read()
        w = {n: raw[model.layout.offsets[n]:model.layout.offsets[n] + math.prod(s) * 2].view(torch.bfloat16)
             .view(*s).float().to(dev) for n, s in model.layout.shapes.items()}
        h = D.rms_norm(x, w["attn_norm"], cfg.norm_eps)
        qkv = h @ w["wqkv"].t()
        q = qkv[:, :model.hq * hd].view(B, model.hq, hd)
        k = qkv[:, model.hq * hd:(model.hq + model.hkv) * hd].view(B, model.hkv, hd)
        v = qkv[:, (model.hq + model.hkv) * hd:].view(B, model.hkv, hd)
        q, k = D.apply_rope(q, cos, sin), D.apply_rope(k, cos, sin)
        kc = model.kv_t[i, 0].float().clone()
        vc = model.kv_t[i, 1].float().clone()
        kc[:, :, pos] = k
        vc[:, :, pos] = v
        a = D.gqa_decode_attention(q, kc, vc, pos + 1)
        x = x + a @ w["wo"].t()
        h = D.rms_norm(x, w["mlp_norm"], cfg.norm_eps)
        x = x + D.silu_mul(h @ w["wgu"].t()) @ w["wd"].t()
    x = D.rms_norm(x, model.final_norm.float(), cfg.norm_eps)
    head = model.head.read().view(torch.bfloat16).view(model.vocab_local, cfg.dim).float().to(dev)
    return x @ head.t()


def smoke(device: int = 0) -> dict:
    """Tiny tiered decode on cuda:0 with the HBM budget below the footprint."""
    if not lib.is_initialized():
        rt.init("hip", host_budget_mb=4096)
    cfg = CONFIGS["small"]
    m = TieredLlama(cfg, batch=4, context=32, max_new_tokens=8, oversub=2.0, device=device, lookahead=1)
    tok = torch.randint(0, cfg.vocab, (4,), device=m.tdev)
    for _ in range(2):
        tok = m.step(tok)
    torch.cuda.synchronize()
    s = lib.stats()
    out = {"tokens": tok.tolist(), "evictions": s["evictions"], "bytes_htd": s["bytes_xfer_htd"],
           "copy_launches": s["copy_kernel_launches"], "plan": m.describe()}
    m.close()
    assert s["bytes_xfer_htd"] > 0, "smoke did not stream any weights"
    return out
