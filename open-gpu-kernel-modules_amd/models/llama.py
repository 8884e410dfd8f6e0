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

Multi-GPU (one process per GPU, RCCL over xGMI), ``parallel=``:

  * ``"tp"`` (default): Megatron tensor parallelism over ``tp_world`` ranks; each
    rank streams only its 1/N of every layer over its own PCIe link and the
    partial outputs are all-reduced (2 per layer).
  * ``"shards"`` (north-star config 4, "peermem-style P2P shards"): every unit
    (weight matrix / LM-head part, in its resting format) is cut into N byte
    shards; rank r owns shard r (preferred on its GPU, or streamed from its host
    DRAM at 2x oversubscription) and the whole unit is all-gathered over xGMI into
    a transient HBM slot right before use, with look-ahead on a side stream
    (parallel/shards.py UnitGather). Each rank decodes its own B/N sequences
    with the full model (ZeRO-3-style inference). The reference's analogue is
    data resident on one processor read by another through remote mapping /
    read duplication (uvm_va_block.c:11660-11664, :5164).
"""
from __future__ import annotations

import collections
import math
import os
import time
from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import rt
from .._native import lib
from ..ops import bf12, dgemm, fused
from ..ops import decode as D
from ..ops.memory import managed_embedding
from ..parallel import comm, tp as tpmod

ALIGN = 4096
# Resting / raw bytes of the lossless formats on random-init N(0, 0.02) weights,
# measured (BENCH_r02 resting_bytes_ratio for rANS; codec tests for BF11 / BF12):
# what a dry-run plan uses instead of packing a layer.
DRY_PACK_RATIO = {"ans": 0.6642, "bf11": 0.70, "bf12": 0.75, "bf16": 1.0}
# Planning rates (per GPU): PCIe host->HBM measured on the box (profiles/), HBM
# read rate of the decode kernels (profiles/r2_dgemm_sweep.txt, 70B shapes).
PLAN_PCIE_GBPS = 56.7
PLAN_HBM_GBPS = 4000.0
# Diagnostics: the host waits for every streamed unit's copies (instead of a
# GPU-side stream dependency).
_HOST_LEASE_WAIT = os.environ.get("OGKM_HOST_LEASE_WAIT", "0") != "0"
_FLOOR_FALLBACK = os.environ.get("OGKM_FLOOR_FALLBACK", "stop")
# planner off: count only the bytes a prefetch moves against the window (1; default
# 0: unit sizes - measured the same on the 70B, 103.4 vs 102.7 tok/s, and a
# larger in-flight share of a small arena streams more)
_WINDOW_MISSING = os.environ.get("OGKM_WINDOW_MISSING", "0") != "0"


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
    # 8 KV heads like the Llama-3 family: tp8 runs one KV head per rank (the
    # per-rank shape of 70B / 405B tp8), for the 8-rank CPU rehearsal
    "small-kv8": LlamaConfig("small-kv8", 1024, 16, 16, 8, 2816, 4096),
}


def _al(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class LayerLayout:
    """Byte offsets of one TP shard's GEMM weights inside a layer buffer (bf16,
    4 KB aligned). Every matrix is stored in the decode GEMM's fragment order
    (ops/dgemm.py: 16x32 MFMA A-tiles), so the kernel streams it - raw or
    packed - with one coalesced 1 KB wave access per tile. The RMSNorm weights
    live in a separate small resident buffer (TieredLlama.norms).

    The FFN matrices are cut into row parts no larger than the attention
    matrices (``unit_bytes``): gate/up part p = [gate rows r0:r1; up rows r0:r1]
    (its SiLU-mul epilogue yields FFN columns r0:r1), down part q = output rows
    n0:n1. Every part is its own streamed unit, so the HBM held by in-flight
    streaming slots (and the bf16 staging buffer of staged formats) is sized by
    the largest part, not by the ~1 GB gate/up matrix."""

    shapes: dict = field(default_factory=dict)
    offsets: dict = field(default_factory=dict)
    roles: dict = field(default_factory=dict)   # "wqkv" | "wo" | "wgu" | "wd" -> its part names
    rows: dict = field(default_factory=dict)    # part name -> (r0, r1) of its role's output rows
    nbytes: int = 0

    @staticmethod
    def _nparts(rows: int, total_bytes: int, target: int) -> int:
        tiles = rows // 16
        for p in range(1, tiles + 1):
            if tiles % p == 0 and total_bytes // p <= target:
                return p
        return tiles

    @staticmethod
    def build(cfg: LlamaConfig, world: int, unit_bytes: Optional[int] = None) -> "LayerLayout":
        hd = cfg.head_dim
        hq, hkv, f = cfg.n_heads // world, cfg.n_kv_heads // world, cfg.ffn_dim // world
        L = LayerLayout()

        def add(role, name, shape, r0, r1):
            L.shapes[name] = shape
            L.offsets[name] = L.nbytes
            L.rows[name] = (r0, r1)
            L.roles.setdefault(role, []).append(name)
            L.nbytes += _al(math.prod(shape) * 2)

        nqkv = (hq + 2 * hkv) * hd
        add("wqkv", "wqkv", (nqkv, cfg.dim), 0, nqkv)
        add("wo", "wo", (cfg.dim, hq * hd), 0, cfg.dim)
        if unit_bytes is None:
            env = os.environ.get("OGKM_UNIT_MB")
            # Floor (OGKM_UNIT_MIN_MB, default 128 MB): every unit costs fixed host
            # work (lease, unpack, GEMM + reduce launches), so small TP shards keep
            # whole matrices as units instead of ~16 MB slivers (70B tp8: 4 units
            # per layer instead of 13).
            floor = int(float(os.environ.get("OGKM_UNIT_MIN_MB", "128")) * 2**20)
            unit_bytes = (int(float(env) * 2**20) if env
                          else max(max(nqkv * cfg.dim, cfg.dim * hq * hd) * 2, floor))
        p = LayerLayout._nparts(f, 2 * f * cfg.dim * 2, unit_bytes)
        per = f // p
        for j in range(p):
            add("wgu", f"wgu.{j}", (2 * per, cfg.dim), j * per, (j + 1) * per)
        q = LayerLayout._nparts(cfg.dim, cfg.dim * f * 2, unit_bytes)
        per = cfg.dim // q
        for j in range(q):
            add("wd", f"wd.{j}", (per, f), j * per, (j + 1) * per)
        return L


class TieredLlama:
    def __init__(self, cfg: LlamaConfig, batch: int, context: int, max_new_tokens: int = 64, oversub: float = 2.0,
                 device: int = 0, tp_rank: int = 0, tp_world: int = 1, seed: int = 0, lookahead: int = 2,
                 hbm_budget: Optional[int] = None, init_std: float = 0.02, verbose: bool = False,
                 packed: bool = True, weight_format: str = "bf11", tiers: str = "host", cxl_frac: float = 0.5,
                 kv_format: str = "bf16", parallel: str = "tp", planner: str = "static",
                 kv_tiering: bool = False, dry_run: bool = False, pack_ratio: Optional[float] = None,
                 attach: Optional[dict] = None):
        """``dry_run``: compute the residency plan only (budget, resident / streamed
        units, per-step traffic: ``traffic()``) - no runtime, no allocation, no
        weights generated; packed formats use ``pack_ratio`` (resting / raw bytes,
        default the measured rANS / BF11 ratios) instead of packing layer 0. Used
        by ``bench.py --plan-only`` for configurations larger than the box.
        ``attach``: resume a saved model (``TieredLlama.restore``) - the managed
        ranges already exist (restored in place from a residency checkpoint with
        data); nothing is generated or written, the position is the saved one."""
        self._ctor = dict(cfg=cfg.name, batch=batch, context=context, max_new_tokens=max_new_tokens, oversub=oversub,
                          device=device, tp_rank=tp_rank, tp_world=tp_world, seed=seed, lookahead=lookahead,
                          hbm_budget=hbm_budget, init_std=init_std, packed=packed, weight_format=weight_format,
                          tiers=tiers, cxl_frac=cxl_frac, kv_format=kv_format, parallel=parallel, planner=planner,
                          kv_tiering=kv_tiering)
        if parallel not in ("tp", "shards"):
            raise ValueError("parallel must be 'tp' or 'shards'")
        # planner "static": the plan below picks resident layers and pins them
        # with lifetime leases. "off": no plan - every weight prefers HBM, none
        # is pinned, each use is a lease (software fault) and the runtime's LRU,
        # prefetch and eviction decide what stays resident.
        if planner not in ("static", "off"):
            raise ValueError("planner must be 'static' or 'off'")
        self.planner = planner
        self.parallel = parallel
        if parallel == "shards":
            # Data parallel over sequences, weights sharded over ranks: the layer
            # math is the single-GPU model (TP world 1) on B / N local sequences.
            if batch % tp_world:
                raise ValueError("shards: the global batch must be a multiple of the rank count")
            self.srank, self.sworld = tp_rank, tp_world
            self.B_global = batch
            batch //= tp_world
            self.b0 = self.srank * batch
            tp_rank, tp_world = 0, 1
        else:
            self.srank, self.sworld, self.B_global, self.b0 = 0, 1, batch, 0
        assert cfg.n_heads % tp_world == 0 and cfg.n_kv_heads % tp_world == 0 and cfg.ffn_dim % tp_world == 0
        assert cfg.vocab % tp_world == 0
        self.cfg, self.B, self.ctx = cfg, batch, context
        self.T = context + max_new_tokens
        self.dev = device
        self.rank, self.world = tp_rank, tp_world
        self.dry_run = dry_run
        self.fake = dry_run or lib.backend_name() == "fake"
        self.tdev = torch.device("cpu") if self.fake else torch.device("cuda", device)
        self.verbose = verbose
        # Fully resident (oversub <= 1): nothing streams, so each role is one
        # unit - one GEMM per role (a gate/up split only pays when streaming).
        whole = oversub <= 1.0 and not os.environ.get("OGKM_UNIT_MB")
        self.layout = LayerLayout.build(cfg, tp_world, unit_bytes=(1 << 62) if whole else None)
        hd = cfg.head_dim
        self.hq, self.hkv = cfg.n_heads // tp_world, cfg.n_kv_heads // tp_world
        self.f_local = cfg.ffn_dim // tp_world
        self.vocab_local = cfg.vocab // tp_world
        # ---- footprint and budget
        self.layer_bytes = self.layout.nbytes
        self.head_bytes = _al(self.vocab_local * cfg.dim * 2)
        self.embed_bytes = _al(cfg.vocab * cfg.dim * 2)
        self.kv_layer_bytes = 2 * batch * self.hkv * self.T * hd * 2
        self.kv_bytes = cfg.n_layers * self.kv_layer_bytes
        self.norm_bytes = _al((2 * cfg.n_layers + 1) * cfg.dim * 2)
        self.footprint = (self.embed_bytes + (cfg.n_layers * self.layer_bytes + self.head_bytes) // self.sworld
                          + self.kv_bytes + self.norm_bytes)
        self.oversub = oversub
        blk = 2 << 20
        budget = hbm_budget if hbm_budget is not None else int(self.footprint / oversub)
        self.budget = budget // blk * blk

        def chunks(n):
            return (n + blk - 1) // blk * blk
        # Weight storage (every matrix in the decode GEMM's fragment order).
        # "bf11": every weight rests packed (lossless BF11, ~0.70x) in whatever
        # tier holds it - host, CXL and HBM - and the decode GEMM reads the packed
        # stream directly (decoded in registers: no bf16 copy exists anywhere).
        # "bf12": packed BF12 (0.75x), unpacked into a bf16 staging buffer
        # right before its layer runs (carved out of the same HBM budget).
        # "bf16": raw weights; with ``packed`` the runtime keeps streamed host
        # copies BF12 and decodes them inside the H2D copy kernel.
        if weight_format not in ("bf11", "bf12", "ans", "bf16"):
            raise ValueError("weight_format must be 'bf11', 'bf12', 'ans' or 'bf16'")
        self.wfmt = weight_format
        self.wpacked = weight_format in ("bf11", "bf12", "ans")   # weights rest packed in every tier
        self.packed = packed and weight_format == "bf16"
        self.staged = weight_format in ("bf12", "ans")
        self.packfmt = "bf11s" if weight_format == "bf11" else weight_format
        unit_raw_max = max(math.prod(sh) * 2 for sh in self.layout.shapes.values())
        self.stage_bytes = chunks(unit_raw_max + (1 << 20)) if self.staged else 0
        # shards: the largest unit's shard (its resting stream is never bigger than
        # the raw bf16 + chunk headers) and the all-gather slots that hold whole units
        self.gather_depth = max(2, int(os.environ.get("OGKM_GATHER_DEPTH", "2")))
        # resting-stream bound of a unit: raw bf16 + chunk headers (packed streams never exceed it)
        stream_bound = unit_raw_max + 8192 + ((unit_raw_max >> 21) + 1) * 1024
        self.shard_max = _al(-(-stream_bound // self.sworld)) if self.sworld > 1 else 0
        self.gather_bytes = chunks(self.gather_depth * self.sworld * self.shard_max) if self.sworld > 1 else 0
        self.arena_bytes = self.budget - self.stage_bytes - self.gather_bytes
        # KV tiering: each layer's prefilled context is a managed
        # unit like a weight matrix - resident with its layer or streamed (and
        # evicted) past the budget, prefetched layer-ahead; decode tokens go to a
        # small always-resident tail. Per layer, prefix + tail are assembled in
        # one [2, B, hkv, T, hd] scratch that attention reads.
        self.kv_tier = bool(kv_tiering)
        self.kv_split = kv_format != "bf16" or self.kv_tier
        if self.kv_split:
            self.arena_bytes -= chunks(self.kv_layer_bytes)  # the per-layer KV scratch
        if self.arena_bytes <= 0:
            raise ValueError(f"HBM budget {self.budget / 2**30:.2f} GiB does not cover the unpack staging "
                             f"({self.stage_bytes / 2**30:.2f} GiB) and all-gather slots "
                             f"({self.gather_bytes / 2**30:.2f} GiB): lower the oversubscription")
        # With the pluggable allocator (config 2) torch tensors - staging,
        # KV scratch, activations - come out of the same HBM arena: the arena is
        # the whole budget and the plan keeps 256 MB of it for activations.
        self.torch_in_arena = False
        if not self.fake:
            from .. import allocator as _alloc
            self.torch_in_arena = _alloc.enabled()
        self.arena_init_bytes = self.budget if self.torch_in_arena else self.arena_bytes
        if self.torch_in_arena:
            self.arena_bytes -= 256 << 20
        if not dry_run and attach is None:  # (restore sizes the arena before loading the checkpoint)
            lib.init_device(device, self.arena_init_bytes)
        if pack_ratio is None:
            pack_ratio = DRY_PACK_RATIO.get(weight_format, 1.0)
        self.pinfo: dict = {}
        self.pmode: dict = {}
        gpu = rt.Loc.gpu(device)
        host = rt.Loc.host(0 if dry_run else None)
        t0 = time.perf_counter()
        self._seed, self._std = seed, init_std
        # ---- KV cache format. "bf16": raw [L, 2, B, hkv, T, hd]. "bf11": the
        # prefilled context rests losslessly packed (one BF11 chunk per (k|v, b,
        # head) row block of ctx x hd values), decode tokens in a raw tail; per
        # layer the prefix is unpacked (k_bf12_unpack, strided into row blocks of
        # T x hd) into one [2, B, hkv, T, hd] scratch that attention reads.
        if kv_format not in ("bf16", "bf11", "ans"):
            raise ValueError("kv_format must be 'bf16', 'bf11' or 'ans'")
        # One (k|v, b, head) row block of the prefilled context = ctx * hd values:
        # one codec chunk, or 2^n chunks of 1 Mi (the largest chunk) for long
        # contexts, unpacked contiguously into the strided cache row.
        rowv = context * hd
        if kv_format != "bf16" and (rowv & (rowv - 1) or rowv < 8192):
            raise ValueError("packed kv_format needs context * head_dim to be a power of two >= 8 Ki")
        cv = min(rowv, 1 << 20)
        self.kv_row_chunks = rowv // cv
        self.kv_format = kv_format
        self.tail = self.T - context
        self.kv_tail_bytes = cfg.n_layers * 2 * batch * self.hkv * self.tail * hd * 2
        self.kv_scratch_bytes = self.kv_layer_bytes if self.kv_split else 0
        self.kv_streams, self.kv_infos, self.kv_slot = [], [], 0
        self.kv_prefix_bytes = 2 * batch * self.hkv * context * hd * 2  # raw bf16 prefix of one layer
        if kv_format != "bf16" and attach is not None:
            self.kv_infos = [bf12.PackedInfo(**d) for d in attach["kv_infos"]]
            self.kv_slot = attach["kv_slot"]
            self.kv_resident_bytes = cfg.n_layers * self.kv_slot + _al(self.kv_tail_bytes)
        elif kv_format != "bf16" and dry_run:
            self.kv_slot = _al(int(self.kv_prefix_bytes * DRY_PACK_RATIO.get(kv_format, 1.0)) + 65536)
            self.kv_resident_bytes = cfg.n_layers * self.kv_slot + _al(self.kv_tail_bytes)
        elif kv_format != "bf16":
            for i, full in enumerate(self._gen_prefill()):
                st, inf = bf12.pack(full, chunk_values=cv, fmt=kv_format)
                self.kv_streams.append(st)
                self.kv_infos.append(inf)
                del full
            self.kv_slot = _al(max(i.nbytes for i in self.kv_infos))
            self.kv_resident_bytes = cfg.n_layers * self.kv_slot + _al(self.kv_tail_bytes)
        else:
            self.kv_resident_bytes = _al(self.kv_bytes)
        if self.kv_tier:
            # prefixes leave the resident range: they are units now
            self.kv_unit_bytes = self.kv_slot if kv_format != "bf16" else _al(self.kv_prefix_bytes)
            self.kv_resident_bytes = _al(self.kv_tail_bytes)
        else:
            self.kv_unit_bytes = 0
        # ---- streamed units: each layer's four matrices and the LM head split
        # into row parts no larger than the largest matrix. Streaming per unit
        # (not per layer) keeps the HBM reserved for in-flight streaming at a
        # few units instead of a few whole layers - those bytes hold resident
        # layers instead, so fewer bytes cross PCIe every step.
        self.parts = tuple(self.layout.shapes)
        part_raw = {n: math.prod(sh) * 2 for n, sh in self.layout.shapes.items()}
        self.head_rows = self._head_split(max(part_raw.values()))
        first_parts = None
        if self.wpacked and attach is not None:  # the saved plan's unit sizes
            self.res_part = dict(attach["res_part"])
            self.res_head_part = list(attach["res_head_part"])
        elif self.wpacked and dry_run:
            ratio = pack_ratio
            self.res_part = {n: _al(int(part_raw[n] * ratio * 1.002) + 4096) for n in self.parts}
            self.res_head_part = [_al(int((r1 - r0) * cfg.dim * 2 * ratio * 1.002) + 8192)
                                  for r0, r1 in self.head_rows]
        elif self.wpacked:
            # Layer 0's packed sizes size the plan (all layers share one distribution).
            first_parts = self._pack_parts(self._gen_layer(0))
            ratio = sum(inf.nbytes for _, inf in first_parts.values()) / sum(part_raw.values())
            self.res_part = {n: _al(int(first_parts[n][1].nbytes * 1.002) + 4096) for n in self.parts}
            self.res_head_part = [_al(int((r1 - r0) * cfg.dim * 2 * ratio * 1.002) + 8192)
                                  for r0, r1 in self.head_rows]
        else:
            self.res_part = {n: _al(b) for n, b in part_raw.items()}
            self.res_head_part = [_al((r1 - r0) * cfg.dim * 2) for r0, r1 in self.head_rows]
        if self.sworld > 1:
            # every rank rests 1/N of each unit: plan (and stream) shard bytes
            self.full_part, self.full_head_part = dict(self.res_part), list(self.res_head_part)
            shard = lambda b: min(self.shard_max, _al(-(-b // self.sworld)))  # noqa: E731
            self.res_part = {n: shard(b) for n, b in self.res_part.items()}
            self.res_head_part = [shard(b) for b in self.res_head_part]
        self.res_layer_bytes = sum(self.res_part.values())
        self.res_head_bytes = sum(self.res_head_part)
        # ---- residency plan (in resting bytes: packed or raw)
        # Streaming slots: the unit in use + `lookahead` prefetched + one
        # run-ahead slot (the host runs ahead of the GPU: when unit u+lookahead is
        # prefetched, unit u-1 may still be read by queued kernels).
        slot = max([chunks(b) for b in self.res_part.values()] + [chunks(b) for b in self.res_head_part]
                   + [chunks(self.kv_unit_bytes)])
        self.slot_bytes = slot
        # The prefetch window must cover the longest resident stretch (~2 layers
        # of compute) or the link idles behind it: at least OGKM_WINDOW_MB in flight.
        # (Capped at a quarter of the arena left after the KV cache: small models.)
        layer_cost = sum(chunks(b) for b in self.res_part.values()) + chunks(self.kv_unit_bytes)
        head_cost = sum(chunks(b) for b in self.res_head_part)
        fixed = chunks(self.kv_resident_bytes + self.norm_bytes)
        # With the KV cache streamed (tiering: a ~1 GB unit per layer at 32k
        # context) and the runtime deciding residency, the host's prefetch calls
        # for those units are long (they evict as much): a window of ~13 KV units
        # keeps the link busy through them (70B, 32k, batch 8: 10.3 tok/s at
        # 56.8 GB/s with 13 units vs 8.1 at 41 with 384 MB; 6-8 units 8.8-10.0,
        # 16 units 9.2-9.3 - the host's prefetch calls grow with the window;
        # profiles/r5_longctx.jsonl).
        wdef = 384 * 2**20
        if self.kv_tier and planner == "off" and self.kv_unit_bytes:
            wdef = max(wdef, 13 * chunks(self.kv_unit_bytes))
        window_min = int(float(os.environ.get("OGKM_WINDOW_MB", "0")) * 2**20) or wdef
        lookahead_arg = lookahead
        lookahead = max(lookahead, min(-(-window_min // slot), max(0, self.arena_bytes - fixed) // (4 * slot)))
        runahead = self.runahead = int(os.environ.get("OGKM_RUNAHEAD", "1"))
        staging = (lookahead + 1 + runahead) * slot
        if self.arena_bytes - fixed - staging < slot:  # tiny budgets: no room for the run-ahead slot
            staging = (lookahead + 1) * slot
        avail = self.arena_bytes - fixed - staging
        if avail < 0:
            raise ValueError(f"HBM budget {self.budget/2**30:.1f} GiB too small for KV + staging "
                             f"({(fixed + staging + self.stage_bytes)/2**30:.1f} GiB)")
        n_res = max(0, min(cfg.n_layers, avail // layer_cost - int(os.environ.get("OGKM_RESIDENT_MARGIN", "0"))))
        # What the static plan would stream per step (planner off: the bytes the
        # runtime's own residency is measured against; traffic() plans with it).
        res_s = [((i + 1) * n_res) // cfg.n_layers > (i * n_res) // cfg.n_layers for i in range(cfg.n_layers)]
        self.plan_streamed_bytes = (sum(self.res_layer_bytes + self.kv_unit_bytes for r in res_s if not r)
                                    + (0 if avail - n_res * layer_cost >= head_cost else self.res_head_bytes))
        if (planner == "off" and n_res == cfg.n_layers and avail - n_res * layer_cost >= head_cost
                and os.environ.get("OGKM_FITS_STATIC", "0") != "0"):
            # (round-4 fallback, now off: with the runtime's resident-extent
            # lease fast path, leasing every unit at every use costs what the
            # lifetime pins did - csrc/core/migrate.cpp fast_lease)
            planner = self.planner = "static"
        if planner == "off":
            n_res, avail = 0, 0
        left = avail - n_res * layer_cost
        self.head_resident = left >= head_cost and planner == "static"
        if self.head_resident:
            left -= head_cost
        # spread resident layers evenly so streaming continues behind them
        self.resident = [((i + 1) * n_res) // cfg.n_layers > (i * n_res) // cfg.n_layers for i in range(cfg.n_layers)]
        # Opt-in (OGKM_UNIT_RESIDENCY=1): the HBM left over after whole layers
        # holds single units of streamed layers, spread evenly over them. Off by
        # default: measured on the 70B bench it removes the arena's slack, the
        # ring then evicts resident units for run-ahead prefetches and they
        # re-stream (123 -> 99 tok/s, evictions +20%).
        self.extra_resident: set = set()
        if os.environ.get("OGKM_UNIT_RESIDENCY", "0") != "0":
            cand = [("layer", i, n) for i in range(cfg.n_layers) if not self.resident[i] for n in self.parts]
            if cand and left > 0:
                want = min(len(cand), int(left // (layer_cost / len(self.parts))) + 1)
                for j in range(want):
                    key = cand[(j * len(cand)) // want]
                    cost = chunks(self.res_part[key[2]])
                    if cost <= left:
                        self.extra_resident.add(key)
                        left -= cost
        self.streamed_bytes = (sum(self.res_layer_bytes + self.kv_unit_bytes for r in self.resident if not r)
                               - sum(self.res_part[k[2]] for k in self.extra_resident)
                               + (0 if self.head_resident else self.res_head_bytes))
        if planner != "off":
            self.plan_streamed_bytes = self.streamed_bytes
        # a window that wraps around a small streamed set would evict units before their use
        self.lookahead = min(lookahead, max(lookahead_arg, self.streamed_bytes // (8 * slot)))
        self.window_bytes = self.lookahead * slot
        # ---- where streamed tensors rest: host DRAM, or split host DRAM / CXL.mem
        # (three-tier: HBM + host + CXL). Streamed tensors are interleaved over
        # the two so every step reads both pools (capacity tiering; both cross
        # the same PCIe link to the GPU).
        if tiers not in ("host", "host+cxl"):
            raise ValueError("tiers must be 'host' or 'host+cxl'")
        self.tiers = tiers
        self.order = ([k for i in range(cfg.n_layers) for n in self.parts
                       for k in ([("layer", i, n)] + ([("kv", i)] if self.kv_tier and n == self.parts[0] else []))]
                      + [("head", j) for j in range(len(self.head_rows))])
        streamed_keys = [k for k in self.order if not self._is_resident(k)]
        self.rest_loc = {}
        cxl_loc = (rt.Loc("cxl", 0) if dry_run else rt.Loc.cxl()) if tiers == "host+cxl" else None
        for j, key in enumerate(streamed_keys):
            to_cxl = cxl_loc is not None and int((j + 1) * cxl_frac) > int(j * cxl_frac)
            self.rest_loc[key] = cxl_loc if to_cxl else host
        self.cxl_streamed_bytes = sum(self._unit_bytes(k) for k, l in self.rest_loc.items()
                                      if l is cxl_loc and cxl_loc is not None)
        if dry_run:
            self.init_seconds = 0.0
            return
        if attach is not None:
            self._attach(attach)
            return
        # ---- allocate + init
        self.embed = rt.malloc_managed(self.embed_bytes, "embed")
        self.embed.set_preferred_location(host)
        self.embed.set_accessed_by(device)
        # KV cache + the RMSNorm weights (tiny) share one resident range
        self.kv = rt.malloc_managed(self.kv_resident_bytes + self.norm_bytes, "kv")
        self.kv.set_preferred_location(gpu)
        self.ubuf: dict = {}
        for i in range(cfg.n_layers):
            if self.wpacked:
                packs = first_parts if i == 0 else self._pack_parts(self._gen_layer(i))
            else:
                flat = self._gen_layer(i)
                packs = {n: (flat[self.layout.offsets[n] // 2:self.layout.offsets[n] // 2
                                  + math.prod(self.layout.shapes[n])].clone(), None) for n in self.parts}
                del flat
            for n in self.parts:
                self._alloc_unit(("layer", i, n), packs[n][0], packs[n][1], gpu, host)
            del packs
        first_parts = None
        head = self._gen_head_rows()
        for j, (r0, r1) in enumerate(self.head_rows):
            part = dgemm.frag_permute(head[r0:r1].contiguous())
            if self.wpacked:
                st, inf = bf12.pack(part, fmt=self.packfmt)
                self._alloc_unit(("head", j), st, inf, gpu, host)
            else:
                self._alloc_unit(("head", j), part, None, gpu, host)
        del head
        if self.kv_tier:
            gen = None if kv_format != "bf16" else self._gen_prefill()
            for i in range(cfg.n_layers):
                key = ("kv", i)
                data = self.kv_streams[i] if kv_format != "bf16" else next(gen).reshape(-1).view(torch.uint8)
                b = rt.malloc_managed(self.kv_unit_bytes, f"kv-{i}", cpu_view=False)
                self._place(b, self._is_resident(key), gpu, self.rest_loc.get(key, host), self.planner)
                b.write(data)
                self.ubuf[key] = b
                del data
            self.kv_streams = []
        self.embed.write(self._gen_embed())
        if not self.fake:
            torch.cuda.synchronize(self.dev)
        # RMSNorm weights of every layer + the final norm (after the KV cache)
        self.kv.write(torch.ones((2 * cfg.n_layers + 1) * cfg.dim, dtype=torch.bfloat16),
                      offset=self.kv_resident_bytes)
        for i, st in enumerate(self.kv_streams):  # (tiering: written to the KV units above)
            self.kv.write(st, offset=i * self.kv_slot)
        self.kv_streams = []
        self._finish_init(fill_prefill=True)
        self.init_seconds = time.perf_counter() - t0
        if verbose:
            self.describe()

    def _finish_init(self, fill_prefill: bool, pos: Optional[int] = None) -> None:
        """Views, leases and the streaming state over the managed ranges (shared
        by a fresh model and one attached to restored ranges)."""
        cfg, batch, context, device = self.cfg, self.B, self.ctx, self.dev
        hd = cfg.head_dim
        self.stage = (torch.empty(self.stage_bytes // 2, dtype=torch.bfloat16, device=self.tdev)
                      if self.staged else None)
        self.cos, self.sin = D.rope_tables(hd, self.T, cfg.rope_theta, self.tdev)
        # KV cache: leased for the model's lifetime (hot, written every step)
        self.kv_lease = self.kv.acquire(device, rt.WRITE)
        self.kv_lease.wait()
        tdev = "cpu" if self.fake else "cuda"
        self.norm_w = rt._tensor_from_ptr(self.kv_lease.dptr + self.kv_resident_bytes, (2 * cfg.n_layers + 1, cfg.dim),
                                          torch.bfloat16, tdev, device)
        self.final_norm = self.norm_w[2 * cfg.n_layers]
        if not self.kv_split:
            kv = self.kv_lease.tensor((cfg.n_layers, 2, batch, self.hkv, self.T, hd), torch.bfloat16)
            if fill_prefill:
                for i, full in enumerate(self._gen_prefill()):
                    kv[i, :, :, :, :context].copy_(full)
                    del full
            self.kv_t = kv
        else:
            self.kv_t = None
            tail_off = 0 if self.kv_tier else cfg.n_layers * self.kv_slot
            self.kv_tail_t = rt._tensor_from_ptr(self.kv_lease.dptr + tail_off,
                                                 (cfg.n_layers, 2, batch, self.hkv, max(self.tail, 1), hd),
                                                 torch.bfloat16, tdev, device)
            self.kv_scratch = torch.empty(2, batch, self.hkv, self.T, hd, dtype=torch.bfloat16, device=self.tdev)
        self.pos = context if pos is None else pos
        # ---- streaming schedule: use order within a step
        self.stream_seq = [k for k in self.order if not self._is_resident(k)]
        self._pf_next = 0           # next index in stream_seq to prefetch (cyclic)
        self._inflight: list = []   # prefetched, not yet consumed
        self._inflight_b: dict = {}  # key -> bytes its prefetch counted against the window
        # streaming diagnostics (bench.py aux "stream_stats"): prefetches issued /
        # refused by the victim floor, uses that found their unit not prefetched,
        # host ms in acquire and in the run-ahead bound's waits
        self.sstats = dict.fromkeys(("prefetched", "refused", "demand", "prefetch_ms", "acquire_ms", "ahead_wait_ms",
                                     "late_uses", "late_mb"), 0)
        self.diag = False  # bench --verbose: also count bytes not yet placed in HBM when a unit is used

        # Next-use hints (planner off): a streamed unit is next used one step
        # later at the same place in the use order, so the runtime can evict
        # in next-use order (Belady, ChunkArena::set_next_use) instead of
        # recency - on a cyclic step larger than HBM, LRU evicts every unit just
        # before its reuse. The runtime itself splits the hinted units into a
        # keep class sized to its arena, spread over the use order, and a
        # stream class evicted first (SpreadPolicy, csrc/core/spread.cpp) -
        # the model passes nothing but the next uses. Op clock = passes *
        # len(stream_seq) + position. Peer shards hint the same way: each rank's
        # shards are used (gathered) in the same cyclic order.
        self.next_use = (self.planner == "off" and os.environ.get("OGKM_NEXT_USE", "1") != "0"
                         and bool(self.stream_seq))
        self._refs: dict = {}  # (unit, dptr, mode) -> WeightRef (_ref)
        self._seq_pos = {k: j for j, k in enumerate(self.stream_seq)}
        self._pass, self._last_pos = 0, -1
        if self.next_use and not self.dry_run:
            lib.reset_op_clock(self.dev)  # our clock restarts at 0 (a previous model's hints are stale)
        # Bounded run-ahead: compute events of streamed units enqueued but maybe
        # not yet run. Leases wait GPU-side, so without a bound the host would
        # prefetch a whole step ahead and the ring would evict (and wait on)
        # chunks whose readers are still queued - the copies then serialise
        # behind compute and the link idles. The host waits for the unit
        # ``max_ahead`` streamed units back instead (OGKM_MAX_AHEAD).
        self._ahead = collections.deque()
        self.max_ahead = int(os.environ.get("OGKM_MAX_AHEAD", "0")) or (self.lookahead + self.runahead)
        # The per-unit protocol (clock, prefetch window, lease, GPU-side wait,
        # next-use hint; release + run-ahead bound) runs natively: two calls
        # per unit instead of ~100 us of Python (csrc/core/unit_stream.cpp).
        # OGKM_NATIVE_UNITS=0: the Python protocol below (diagnostics use it).
        self._us = None
        if (self.sworld <= 1 and self.stream_seq and not self.dry_run
                and os.environ.get("OGKM_NATIVE_UNITS", "1") != "0"):
            self._us = lib.UnitStream(device, [self._buf(k).id for k in self.stream_seq], self.window_bytes,
                                      self.next_use, 0 if self.fake else self.max_ahead)
        self._raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        self._views: dict = {}
        self.byte_trace = None     # diagnostics: {key: H2D bytes submitted around its use}
        self.use_trace = None      # diagnostics: [(key, acquire s, wait s)] per streamed use
        self._pinned: dict = {}    # resident tensors: key -> weight refs (leased for the model's lifetime)
        self._pin_leases: list = []
        self._kv_pinned: dict = {}  # kv tiering: resident layers' prefix pointers
        self.keep_logits = False   # tests: keep the full-vocab logits of the last step
        # deferred GEMM epilogues in the next launch (step(); OGKM_FUSE_EPI=0: separate reduces)
        self.fuse_epilogues = os.environ.get("OGKM_FUSE_EPI", "1") != "0"
        # fragment-ordered GEMM activations (OGKM_XFRAG=0: row-major)
        self.x_frag = os.environ.get("OGKM_XFRAG", "1") != "0"
        self._xrows = None
        self.last_logits = None
        self.gather = None
        self.gather_cache_bytes = 0
        if self.sworld > 1:
            from ..parallel.shards import UnitGather
            self.gather = UnitGather([k for k in self.order if k[0] != "kv"], self._buf, self._unit_bytes, self.sworld, self.gather_depth,
                                     device=self.tdev, dev_index=device)
            self._gather_cache_setup()
        self._settle()

    def _gather_cache_setup(self) -> None:
        """Shards mode with HBM to spare: whole gathered units kept as read
        duplicates in a managed buffer leased for the model's lifetime (so the
        runtime's arena accounts for them), chosen evenly over the use order;
        they are all-gathered once and then read in place - the reference's
        read duplication of data resident on another processor
        (uvm_va_block.c:5164), sized to what the budget leaves after this
        rank's shards, the resident KV and the streaming window.
        OGKM_GATHER_CACHE_MB: 0 = off, N = at most N MB (default: auto)."""
        from ..parallel import comm
        self._gcache, self._gcache_lease, self.gather_cache_bytes = None, None, 0
        cap_env = os.environ.get("OGKM_GATHER_CACHE_MB")
        if cap_env == "0":
            return
        keys = self.gather.order
        full = {k: _al(self._unit_bytes(k) * self.sworld) for k in keys}
        shards = sum(self._unit_bytes(k) for k in keys)
        spare = (self.arena_bytes - self.kv_resident_bytes - self.norm_bytes - shards - self.window_bytes
                 - 2 * self.slot_bytes)
        if cap_env:
            spare = min(spare, int(float(cap_env) * 2**20))
        # the same choice on every rank: it decides which collectives run
        spare = -comm.max_over_ranks(-float(spare))
        total = sum(full.values())
        if spare < min(full.values()):
            return
        frac = min(1.0, spare / total)
        chosen, used = [], 0
        for j, k in enumerate(keys):  # evenly spread: floor((j + 1) f) > floor(j f)
            if int((j + 1) * frac) > int(j * frac) and used + full[k] <= spare:
                chosen.append(k)
                used += full[k]
        if not chosen:
            return
        self._gcache = rt.malloc_managed(used, "gather_cache")
        self._gcache_lease = self._gcache.acquire(self.dev, rt.WRITE)
        self._gcache_lease.wait()
        buf = self._gcache_lease.tensor((used,), torch.uint8)
        offs, o = {}, 0
        for k in chosen:
            offs[k] = o
            o += full[k]
        self.gather.set_cache(buf, offs)
        self.gather_cache_bytes = used

    # ------------------------------------------------------------------ save / resume
    def save(self, path: str) -> dict:
        """Checkpoint the model mid-decode: the runtime's residency map WITH data
        (every managed range - weights in their resting format, KV cache, norms -
        with its residency, policies, id and VAs; the rings are quiesced first,
        the uvm_suspend analog) plus a JSON sidecar: construction arguments,
        decode position and the unit -> range-id table. ``restore`` resumes it in
        a fresh process in place (same ids and VAs)."""
        import dataclasses
        import json
        from .. import checkpoint
        if not self.fake:
            torch.cuda.synchronize(self.dev)
        checkpoint.save(path + ".rmap", with_data=True)
        side = {"ctor": self._ctor, "pos": self.pos, "embed": self.embed.id, "kv": self.kv.id,
                "units": [[list(k), b.id] for k, b in self.ubuf.items()],
                "pinfo": [[list(k), dataclasses.asdict(v)] for k, v in self.pinfo.items()],
                "pmode": [[list(k), v] for k, v in self.pmode.items()],
                "res_part": self.res_part, "res_head_part": self.res_head_part,
                "kv_infos": [dataclasses.asdict(i) for i in getattr(self, "kv_infos", [])],
                "kv_slot": getattr(self, "kv_slot", 0)}
        with open(path, "w") as f:
            json.dump(side, f)
        return side

    @staticmethod
    def restore(path: str, verbose: bool = False) -> "TieredLlama":
        """Resume a model saved by ``save`` in this (fresh) process: the ranges
        come back under their recorded ids and VAs with their data
        (checkpoint.load in place), then the model attaches to them - nothing is
        regenerated; the next step continues at the saved position."""
        import json
        from .. import checkpoint
        with open(path) as f:
            side = json.load(f)
        kw = dict(side["ctor"])
        cfg = CONFIGS[kw.pop("cfg")]
        # the saved plan's HBM arena first, so the data lands where it was
        plan = TieredLlama(cfg, dry_run=True, pack_ratio=1.0, attach=None, **kw)
        lib.init_device(kw["device"], plan.arena_init_bytes)
        checkpoint.load(path + ".rmap", with_data=True, in_place=True)
        for rid in lib.range_ids():  # shards read duplicates: rebuilt from the shards, not restored
            if lib.range_info(rid)["name"] == "gather_cache":
                rt.ManagedBuffer(rid).free()
        return TieredLlama(cfg, verbose=verbose, attach=side, **kw)

    def _attach(self, side: dict) -> None:
        tup = lambda k: tuple(k)  # noqa: E731 - JSON lists back to unit keys
        self.embed = rt.ManagedBuffer(side["embed"])
        self.kv = rt.ManagedBuffer(side["kv"])
        self.ubuf = {tup(k): rt.ManagedBuffer(i) for k, i in side["units"]}
        self.pinfo = {tup(k): bf12.PackedInfo(**v) for k, v in side["pinfo"]}
        self.pmode = {tup(k): v for k, v in side["pmode"]}
        self.kv_streams = []
        self._finish_init(fill_prefill=False, pos=side["pos"])
        self.init_seconds = 0.0

    def _settle(self) -> None:
        """Bring the residency to its steady state before the first step: the
        planned-resident units take their lifetime leases now (the load's
        writes may have left some of them in host DRAM, evicted by later
        writes) and the first streaming window is prefetched - so step 0 costs
        what every later step does instead of paying the layout's convergence
        (70B tp8 shard: step 0 was 1.86x a steady step)."""
        if self.gather is None:
            for key in self.order:
                if self._is_resident(key) and key not in self._pinned and \
                        not (key[0] == "kv" and key[1] in self._kv_pinned):
                    self._pin_resident(key)
        self._prefetch_ahead()
        if os.environ.get("OGKM_WARM_STEP", "1") != "0":
            # One warm-up decode at load, then the position rewinds (the next
            # step rewrites the same KV slot): kernels are loaded, the compute
            # path's torch allocations are pooled and the streaming cursor sits
            # where every later step finds it - what a serving engine's start-up
            # warm-up does. Step 0 of a run then costs what step 1 does.
            tok = torch.zeros(self.B, dtype=torch.int64, device=self.tdev)
            pos = self.pos
            self.step(tok)
            self.reset(pos)
        if not self.fake:
            torch.cuda.synchronize(self.dev)

    def _pin_resident(self, key):
        """Lifetime lease of a planned-resident unit: later uses cost no
        runtime call. Returns its WeightRef (a KV prefix: its device pointer)."""
        lease = self._buf(key).acquire(self.dev, rt.READ)
        lease.wait(0 if (self.fake or _HOST_LEASE_WAIT) else None)
        self._pin_leases.append(lease)
        if key[0] == "kv":
            self._kv_pinned[key[1]] = lease.dptr
            return lease.dptr
        refs = self._ref(key, lease.dptr, self.pmode.get(key, dgemm.MODE_RAW))
        self._pinned[key] = refs
        return refs

    # ------------------------------------------------------------------ setup
    def describe(self) -> dict:
        d = {
            "model": self.cfg.name, "tp": f"{self.rank}/{self.world}", "parallel": self.parallel,
            "planner": self.planner, "kv_tiering": self.kv_tier,
            "shard": f"{self.srank}/{self.sworld}", "batch": self.B, "global_batch": self.B_global,
            "gather_gb": self.gather_bytes / 1e9, "context": self.ctx,
            "footprint_gb": self.footprint / 1e9, "hbm_budget_gb": self.budget / 1e9,
            "oversubscription": self.footprint / self.budget, "kv_gb": self.kv_bytes / 1e9,
            "layer_gb": self.layer_bytes / 1e9, "resident_layers": sum(self.resident),
            "extra_resident_units": len(self.extra_resident),
            "streamed_layers": self.cfg.n_layers - sum(self.resident), "head_resident": self.head_resident,
            "streamed_gb_per_step": self.plan_streamed_bytes / 1e9, "init_s": getattr(self, "init_seconds", None),
            "packed_host_copies": getattr(self, "packed", False),
            "weight_format": self.wfmt, "resting_layer_gb": self.res_layer_bytes / 1e9,
            "stage_gb": self.stage_bytes / 1e9, "tiers": self.tiers, "kv_format": self.kv_format,
            "kv_resident_gb": self.kv_resident_bytes / 1e9,
            "cxl_streamed_gb_per_step": self.cxl_streamed_bytes / 1e9,
            "stream_slot_gb": self.slot_bytes / 1e9, "head_parts": len(self.head_rows),
        }
        if getattr(self, "ubuf", None) and getattr(self, "kv", None) is not None:
            # what the runtime really holds (packed where packed) per HBM byte
            resting = sum(b.size for b in self.ubuf.values()) + self.kv.size + self.embed.size
            d["resting_gb"] = resting / 1e9
            d["physical_oversubscription"] = resting / self.budget
        else:
            d["physical_oversubscription"] = d["oversubscription"]
        if self.verbose and self.rank == 0:
            print("[ogkm] plan:", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}, flush=True)
        return d

    def traffic(self) -> dict:
        """Per-rank, per-step traffic this plan implies, and the time it predicts.
          pcie_gb:  streamed units (host / CXL -> HBM over this GPU's PCIe link)
          xgmi_gb:  bytes this rank receives over the links - tp: 2 ring
                    all-reduces of the [B, dim] bf16 activations per layer
                    (2 (W-1)/W each) + the vocab-argmax gather; shards: every
                    unit all-gathered each step, (W-1) shards of it
          hbm_gb:   weight + KV bytes the kernels read from HBM (staged formats:
                    packed read + bf16 write + bf16 read)
        predicted_ms = max(PCIe, HBM) time + the tp collectives' latency-bound
        time (on the critical path), or max(PCIe, HBM, all-gather) for shards
        (gathers run ahead on a side stream)."""
        from ..parallel import topology
        cfg, W = self.cfg, max(self.world, self.sworld)
        n_units = len(self.order)
        pcie = self.plan_streamed_bytes
        if self.sworld > 1:
            shard = sum(self._unit_bytes(k) for k in self.order if k[0] != "kv")
            xgmi = (self.sworld - 1) * shard
            full = {k: self._unit_bytes(k) * self.sworld for k in self.order if k[0] != "kv"}
            topo = topology.PeerTopology(self.sworld)
            xgmi_s = sum(topo.allgather_seconds(b, self.sworld, "direct") for b in full.values())
            n_coll = len(full)
        elif self.world > 1:
            act = self.B * cfg.dim * 2
            n_coll = 2 * cfg.n_layers + 1
            xgmi = 2 * cfg.n_layers * 2 * (self.world - 1) / self.world * act + (self.world - 1) * self.B * 2 * 4
            lat = topology.COLLECTIVE_LATENCY_US * 1e-6
            xgmi_s = n_coll * lat + xgmi / (topology.XGMI_LINK_GBPS * 1e9)
        else:
            xgmi, xgmi_s, n_coll = 0, 0.0, 0
        resting = self.res_layer_bytes * cfg.n_layers + self.res_head_bytes
        raw = self.layer_bytes * cfg.n_layers + self.head_bytes
        if self.sworld > 1:  # every rank runs the whole model on gathered units
            resting, raw = resting * self.sworld, raw
        weights_hbm = resting + 2 * raw if self.staged else (resting if self.wpacked else raw)
        kv_read = self.kv_bytes * (self.ctx + 1) / self.T
        hbm = weights_hbm + kv_read
        pcie_s, hbm_s = pcie / (PLAN_PCIE_GBPS * 1e9), hbm / (PLAN_HBM_GBPS * 1e9)
        pred = max(pcie_s, hbm_s, xgmi_s) if self.sworld > 1 else max(pcie_s, hbm_s) + xgmi_s
        return {"pcie_gb": pcie / 1e9, "xgmi_gb": xgmi / 1e9, "hbm_gb": hbm / 1e9, "collectives": n_coll,
                "pcie_ms": pcie_s * 1e3, "xgmi_ms": xgmi_s * 1e3, "hbm_ms": hbm_s * 1e3,
                "predicted_ms": pred * 1e3, "units": n_units, "world": W}

    def _is_resident(self, key) -> bool:
        if key[0] == "layer":
            return self.resident[key[1]] or key in self.extra_resident
        if key[0] == "kv":
            return self.resident[key[1]]
        return self.head_resident

    def _buf(self, key) -> "rt.ManagedBuffer":
        return self.ubuf[key]

    def _unit_bytes(self, key) -> int:
        if key[0] == "kv":
            return self.kv_unit_bytes
        return self.res_part[key[2]] if key[0] == "layer" else self.res_head_part[key[1]]

    def _unit_shape(self, key) -> tuple:
        if key[0] == "layer":
            return self.layout.shapes[key[2]]
        r0, r1 = self.head_rows[key[1]]
        return (r1 - r0, self.cfg.dim)

    def _head_split(self, max_part_bytes: int) -> list:
        """Row ranges (multiples of 16) splitting the LM head into parts of at
        most ~max_part_bytes of bf16."""
        rows = self.vocab_local
        row_bytes = self.cfg.dim * 2
        n = max(1, -(-rows * row_bytes // max_part_bytes))
        per = -(-rows // n)
        per = -(-per // 16) * 16
        out, r = [], 0
        while r < rows:
            out.append((r, min(rows, r + per)))
            r += per
        return out

    def _pack_parts(self, flat: torch.Tensor) -> dict:
        """Split a layer's flat fragment-ordered weights into its matrices and
        pack each one (its own BF11/BF12 stream)."""
        out = {}
        for n in self.parts:
            off = self.layout.offsets[n] // 2
            out[n] = bf12.pack(flat[off:off + math.prod(self.layout.shapes[n])], fmt=self.packfmt)
        return out

    def _alloc_unit(self, key, data: torch.Tensor, info, gpu, host) -> None:
        name = "-".join(str(x) for x in key)
        resident = self._is_resident(key)
        if self.sworld > 1:
            # bytes [r S, (r+1) S) of the unit's resting stream (zero padded)
            S = self._unit_bytes(key)
            raw = data.reshape(-1).contiguous().cpu().view(torch.uint8)
            part = torch.zeros(S, dtype=torch.uint8)
            lo = min(raw.numel(), self.srank * S)
            hi = min(raw.numel(), lo + S)
            part[:hi - lo] = raw[lo:hi]
            if raw.numel() > self.sworld * S:
                raise ValueError(f"unit {key} does not fit {self.sworld} shards of {S} bytes")
            b = rt.malloc_managed(S, name, cpu_view=False)
            if info is not None:
                self.pinfo[key] = info
                self.pmode[key] = dgemm.packed_mode(data) if not self.staged else dgemm.MODE_RAW
            self._place(b, resident, gpu, self.rest_loc.get(key, host), self.planner)
            b.write(part)
            self.ubuf[key] = b
            return
        if info is not None:
            b = rt.malloc_managed(info.nbytes, name, cpu_view=False)
            self.pinfo[key] = info
            self.pmode[key] = dgemm.packed_mode(data) if not self.staged else dgemm.MODE_RAW
        else:
            b = rt.malloc_managed(data.numel() * 2, name, packed_bf16=self.packed and not resident)
        self._place(b, resident, gpu, self.rest_loc.get(key, host), self.planner)
        b.write(data)
        self.ubuf[key] = b

    @staticmethod
    def _place(b, resident: bool, gpu, host, planner: str = "static") -> None:
        if planner == "off":
            # no plan: HBM preferred, read-duplicated (an eviction drops the HBM
            # copy, the host copy stays) - residency is the runtime's decision
            b.set_preferred_location(gpu)
            b.set_read_mostly(True)
        elif resident:
            b.set_preferred_location(gpu)
        else:
            b.set_preferred_location(host)
            b.set_read_mostly(True)

    def _gen_layer(self, i: int) -> torch.Tensor:
        """Layer i's weights (this TP rank's shard) in the LayerLayout, as a flat
        bf16 tensor of layer_bytes / 2 values (random init, deterministic)."""
        cfg, L = self.cfg, self.layout
        hd = cfg.head_dim
        dev, std = self.tdev, self._std
        flat = torch.zeros(self.layer_bytes // 2, dtype=torch.bfloat16, device=dev)

        def put(name, t):
            off = L.offsets[name] // 2
            flat[off:off + t.numel()].copy_(dgemm.frag_permute(t.contiguous()))

        g = torch.Generator(device=dev).manual_seed(self._seed * 1000003 + i)
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
        wg, wu = tpmod.shard_rows(wg, self.rank, self.world), tpmod.shard_rows(wu, self.rank, self.world)
        for name in L.roles["wgu"]:
            r0, r1 = L.rows[name]
            put(name, torch.cat([wg[r0:r1], wu[r0:r1]], 0))
        del wg, wu
        wd = torch.empty(cfg.dim, cfg.ffn_dim, dtype=torch.bfloat16, device=dev).normal_(0, std, generator=g)
        wd = tpmod.shard_cols(wd, self.rank, self.world)
        for name in L.roles["wd"]:
            r0, r1 = L.rows[name]
            put(name, wd[r0:r1])
        del wd
        return flat

    def _gen_prefill(self):
        """Synthetic prefilled context per layer, [2, B, hkv, ctx, hd] bf16,
        generated at full head count and sliced to this rank's KV heads so every
        TP degree decodes the same model state."""
        cfg = self.cfg
        g = torch.Generator(device=self.tdev).manual_seed(self._seed + 7919)
        h0 = self.rank * self.hkv
        for _ in range(cfg.n_layers):
            full = torch.empty(2, self.B_global, cfg.n_kv_heads, self.ctx, cfg.head_dim, dtype=torch.bfloat16,
                               device=self.tdev)
            full.normal_(0.0, 1.0, generator=g)
            yield full[:, self.b0:self.b0 + self.B, h0:h0 + self.hkv].contiguous()
            del full

    def _kv_layer(self, i: int, pos: int) -> torch.Tensor:
        """Layer i's KV cache as [2, B, hkv, T, hd], valid for positions < pos."""
        if not self.kv_split:
            return self.kv_t[i]
        sc = self.kv_scratch
        lease, ptr = self._kv_prefix(i) if self.kv_tier else (None, self.kv_lease.dptr + i * self.kv_slot)
        if self.kv_format != "bf16":
            bf12.unpack_into(sc, ptr, self.kv_infos[i], self.dev, 0 if self.fake else None,
                             dst_stride=self.T * self.cfg.head_dim, row_chunks=self.kv_row_chunks)
        else:
            hd = self.cfg.head_dim
            pre = rt._tensor_from_ptr(ptr, (2, self.B, self.hkv, self.ctx, hd), torch.bfloat16,
                                      "cpu" if self.fake else "cuda", self.dev)
            sc[:, :, :, :self.ctx].copy_(pre)
        if isinstance(lease, tuple):  # native unit protocol: release + run-ahead bound in one call
            self._us.release(lease[1], self._stream_handle(), not self.fake)
        elif lease is not None:  # the prefix's readers are enqueued: the unit may be evicted behind them
            lease.release(0 if self.fake else None)
            self._mark_consumed()
        t = pos - self.ctx
        if t > 0:
            sc[:, :, :, self.ctx:pos].copy_(self.kv_tail_t[i, :, :, :, :t])
        return sc

    def _rope_append(self, i: int, pos: int, kv_layer: torch.Tensor, qkv: torch.Tensor) -> torch.Tensor:
        """RoPE on q/k + append k/v at pos (into the cache / scratch and the
        packed cache's raw tail) in one fused kernel; returns rotated q."""
        tail = self.kv_tail_t[i] if self.kv_split else None
        return fused.rope_kv(qkv, self.cos[pos], self.sin[pos], kv_layer, pos, self.hq, self.hkv, tail=tail,
                             tail_pos=pos - self.ctx, device_index=self.dev)

    def host_kv(self, i: int) -> torch.Tensor:
        """Layer i's KV cache [2, B, hkv, T, hd] on the host (reference numerics)."""
        if not self.kv_split:
            return self.kv_t[i].to("cpu", copy=True)
        if not self.fake:
            torch.cuda.synchronize(self.dev)
        src, off = (self.ubuf[("kv", i)], 0) if self.kv_tier else (self.kv, i * self.kv_slot)
        out = torch.zeros(2, self.B, self.hkv, self.T, self.cfg.head_dim, dtype=torch.bfloat16)
        if self.kv_format != "bf16":
            raw = src.read(offset=off, nbytes=self.kv_infos[i].nbytes)
            pre = bf12.unpack_host(raw, self.kv_infos[i]).view(2, self.B, self.hkv, self.ctx, self.cfg.head_dim)
        else:
            raw = src.read(offset=off, nbytes=self.kv_prefix_bytes)
            pre = raw.view(torch.bfloat16).view(2, self.B, self.hkv, self.ctx, self.cfg.head_dim)
        out[:, :, :, :self.ctx] = pre
        out[:, :, :, self.ctx:] = self.kv_tail_t[i, :, :, :, :self.tail].cpu()
        return out

    def _head_gen(self) -> torch.Generator:
        return torch.Generator(device=self.tdev).manual_seed(self._seed * 1000003 + 999983)

    def _gen_embed(self) -> torch.Tensor:
        cfg = self.cfg
        return torch.empty(cfg.vocab, cfg.dim, dtype=torch.bfloat16, device=self.tdev).normal_(
            0, 1.0, generator=self._head_gen())

    def _gen_head_rows(self) -> torch.Tensor:
        """This rank's LM-head rows [vocab_local, dim] (row-major, not permuted)."""
        cfg = self.cfg
        g = self._head_gen()
        torch.empty(cfg.vocab, cfg.dim, dtype=torch.bfloat16, device=self.tdev).normal_(0, 1.0, generator=g)  # embed draw
        head = torch.empty(cfg.vocab, cfg.dim, dtype=torch.bfloat16, device=self.tdev).normal_(0, self._std, generator=g)
        return tpmod.shard_rows(head, self.rank, self.world).contiguous()

    def host_weights(self, key) -> torch.Tensor:
        """The bf16 values of one unit as stored (unpacked on the host, still in
        fragment order) - for reference numerics."""
        raw = self._buf(key).read()
        if self.wpacked:
            return bf12.unpack_host(raw, self.pinfo[key])
        return raw.view(torch.bfloat16)

    def host_matrix(self, key) -> torch.Tensor:
        """One weight matrix as a plain [N, K] bf16 CPU tensor (reference numerics):
        key ("layer", i, name), ("head", j) or ("head",) for the whole LM head."""
        if key == ("head",):
            return torch.cat([self.host_matrix(("head", j)) for j in range(len(self.head_rows))])
        if key[0] == "layer" and key[2] not in self.layout.shapes:  # a whole role: reassemble its parts
            mats = [self.host_matrix(("layer", key[1], n)) for n in self.layout.roles[key[2]]]
            if key[2] == "wgu":
                return torch.cat([m[:m.shape[0] // 2] for m in mats] + [m[m.shape[0] // 2:] for m in mats])
            return torch.cat(mats)
        n, k = self._unit_shape(key)
        return dgemm.frag_unpermute(self.host_weights(key)[:n * k], n, k)

    # ------------------------------------------------------------------ streaming
    def _due(self, key) -> int:
        """Op-clock time of the next use of streamed unit ``key``."""
        p = self._seq_pos[key]
        return (self._pass + (p <= self._last_pos)) * len(self.stream_seq) + p

    def _clock_use(self, key) -> None:
        """Next-use mode: advance the op clock to ``key``'s use."""
        p = self._seq_pos.get(key)
        if p is None:
            return
        if p <= self._last_pos:
            self._pass += 1
        self._last_pos = p
        lib.set_op_clock(self.dev, self._pass * len(self.stream_seq) + p)

    def _hint_used(self, key) -> None:
        """Next-use mode, once ``key`` is leased: its next use is one pass later
        (hinted after the lease pinned it - before, the prefetches queued for
        this use would see it as the furthest-needed unit and evict it). The
        runtime decides the unit's keep / stream class from these hints."""
        if key in self._seq_pos:
            n = len(self.stream_seq)
            p = self._seq_pos[key]
            self._buf(key).hint_next_use(self._pass * n + p + n)

    def _native(self) -> bool:
        """Native unit protocol in use (not when a diagnostic needs the Python one)."""
        return self._us is not None and not (self.diag or self.byte_trace is not None or self.use_trace is not None)

    def _stream_handle(self) -> int:
        if self.fake:
            return 0
        if self._raw_stream is not None:
            return self._raw_stream(self.dev)
        return torch.cuda.current_stream(self.dev).cuda_stream

    def stream_stats(self) -> dict:
        """Streaming counters (bench.py aux stream_stats): prefetches issued /
        refused by the victim floor, uses not prefetched, host ms in prefetch /
        acquire / the run-ahead bound."""
        out = dict(self.sstats)
        if self._us is not None:
            for k, v in self._us.stats().items():
                out[k] = out.get(k, 0) + v
        return out

    def reset_stream_stats(self) -> None:
        self.sstats = dict.fromkeys(self.sstats, 0)
        if self._us is not None:
            self._us.reset_stats()

    def _prefetch_ahead(self) -> None:
        """Keep up to ``window_bytes`` of upcoming streamed tensors in flight on the ring."""
        if not self.stream_seq:
            return
        if self._native():
            self._us.prefetch_window()
            return
        inflight = sum(self._inflight_b.get(k, 0) for k in self._inflight)
        n = len(self.stream_seq)
        while len(self._inflight) < n:
            key = self.stream_seq[self._pf_next]
            buf = self._buf(key)
            nb = buf.size
            if self.next_use and _WINDOW_MISSING:
                # next-use mode keeps part of the units resident: the window
                # is the bytes in flight on the link, not the units ahead
                nb -= buf.resident_bytes(rt.Loc.gpu(self.dev))
            if self._inflight and inflight + nb > self.window_bytes:
                break
            t_pf = time.perf_counter()
            if self.next_use:
                # evict only units needed after this one; refused (no such
                # window): OGKM_FLOOR_FALLBACK=stop leaves it to its use,
                # =plain prefetches it anyway (recency / next-use order without
                # the floor, as the fault at its use would)
                try:
                    self._buf(key).prefetch(rt.Loc.gpu(self.dev), needed_at=self._due(key))
                except lib.RuntimeStatusError:
                    self.sstats["refused"] += 1
                    if _FLOOR_FALLBACK != "plain":
                        break
                    self._buf(key).prefetch(rt.Loc.gpu(self.dev))
            else:
                self._buf(key).prefetch(rt.Loc.gpu(self.dev))
            self.sstats["prefetch_ms"] += (time.perf_counter() - t_pf) * 1e3
            self._inflight.append(key)
            self.sstats["prefetched"] += 1
            self._inflight_b[key] = nb
            inflight += nb
            self._pf_next = (self._pf_next + 1) % n

    def _use(self, key):
        """Fault one unit in (lease) and return (lease or None, its WeightRef).
        bf11: the GEMM reads the packed stream in place (the lease is held until
        it is enqueued). bf12 / ans: the stream is unpacked into the staging
        buffer on the compute stream and the lease is released right away (the
        ring reuses the chunks only after the unpack has read them)."""
        if self.gather is not None:
            return self._use_gathered(key)
        pin = self._pinned.get(key)
        if pin is None and self._is_resident(key):
            pin = self._pin_resident(key)
        if pin is not None:  # resident tensor: long-lived lease taken at init, refs cached
            return None, (self._unstage(key, pin.ptr) if self.staged else pin)
        if self._native() and key in self._seq_pos:
            stream = self._stream_handle()
            lid, dptr = self._us.use(self._seq_pos[key], stream, not self.fake)
            if self.staged:
                st = self._unstage(key, dptr)
                self._us.release(lid, stream, not self.fake)
                return None, st
            return ("native", lid), self._ref(key, dptr, self.pmode.get(key, dgemm.MODE_RAW))
        acct = self.byte_trace is not None
        if acct:
            b0 = lib.stats()["bytes_xfer_htd"]
        if not self._is_resident(key):
            if self._inflight and self._inflight[0] == key:
                self._inflight.pop(0)
            else:
                self.sstats["demand"] += 1
            if self.next_use:
                self._clock_use(key)
            self._prefetch_ahead()
        if self.diag and not self.fake:
            miss = self._buf(key).size - self._buf(key).resident_bytes(rt.Loc.gpu(self.dev))
            if miss > 0:
                self.sstats["late_uses"] += 1
                self.sstats["late_mb"] += miss / 2**20
        t_a = time.perf_counter()
        lease = self._buf(key).acquire(self.dev, rt.READ)
        self.sstats["acquire_ms"] += (time.perf_counter() - t_a) * 1e3
        if self.next_use:
            self._hint_used(key)
        if acct:  # H2D bytes submitted while servicing this tensor (prefetch window + its own faults)
            self.byte_trace[key] = self.byte_trace.get(key, 0) + lib.stats()["bytes_xfer_htd"] - b0
        t_w = time.perf_counter()
        lease.wait(0 if (self.fake or _HOST_LEASE_WAIT) else None)
        if self.use_trace is not None:
            self.use_trace.append((key, t_w - t_a, time.perf_counter() - t_w))
        mode = self.pmode.get(key, dgemm.MODE_RAW)
        refs = self._ref(key, lease.dptr, mode)
        if self.staged:
            st = self._unstage(key, lease.dptr)
            lease.release(0 if self.fake else None)
            self._mark_consumed()
            return None, st
        return lease, refs

    def _kv_prefix(self, i: int):
        """Fault layer i's KV prefix unit in: (lease or None, device pointer).
        Resident layers keep theirs leased for the model's lifetime."""
        key = ("kv", i)
        ptr = self._kv_pinned.get(i)
        if ptr is None and self._is_resident(key):
            ptr = self._pin_resident(key)
        if ptr is not None:
            return None, ptr
        if self._native() and key in self._seq_pos:
            lid, dptr = self._us.use(self._seq_pos[key], self._stream_handle(), not self.fake)
            return ("native", lid), dptr
        if not self._is_resident(key):
            if self._inflight and self._inflight[0] == key:
                self._inflight.pop(0)
            if self.next_use:
                self._clock_use(key)
            self._prefetch_ahead()
        lease = self._buf(key).acquire(self.dev, rt.READ)
        if self.next_use:
            self._hint_used(key)
        lease.wait(0 if (self.fake or _HOST_LEASE_WAIT) else None)
        return lease, lease.dptr

    def _mark_consumed(self) -> None:
        """A streamed unit's readers are enqueued: remember where the compute
        stream is, then keep the host at most max_ahead streamed units ahead."""
        if self.fake:
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        self._ahead.append(ev)
        while len(self._ahead) > self.max_ahead:
            t0 = time.perf_counter()
            self._ahead.popleft().synchronize()
            self.sstats["ahead_wait_ms"] += (time.perf_counter() - t0) * 1e3

    def _use_gathered(self, key):
        """shards: fault this rank's shard in (the runtime prefetches streamed
        shards ahead on the ring), all-gather the whole unit over RCCL (issued
        ahead on the gather stream) and return its WeightRef in the gather slot."""
        if not self._is_resident(key):
            if self._inflight and self._inflight[0] == key:
                self._inflight.pop(0)
            if self.next_use:
                self._clock_use(key)
            self._prefetch_ahead()
        full = self.gather.get(key)
        if self.next_use:
            self._hint_used(key)  # this rank's shard: read by the gather just issued
        if self.staged:
            ref = self._unstage(key, full.data_ptr())
            self.gather.done(key)
            self._mark_consumed()
            return None, ref
        return ("gather", key), self._ref(key, full.data_ptr(), self.pmode.get(key, dgemm.MODE_RAW))

    def _unstage(self, key, packed_ptr: int) -> "dgemm.WeightRef":
        """Unpack a packed unit into the bf16 staging buffer (compute stream)."""
        bf12.unpack_into(self.stage, packed_ptr, self.pinfo[key], self.dev, 0 if self.fake else None)
        return self._ref(key, self.stage.data_ptr(), dgemm.MODE_RAW)

    def _ref(self, key, ptr: int, mode: int) -> "dgemm.WeightRef":
        # A unit that stays resident comes back at the same address every step:
        # its WeightRef is built once (host time per unit use is the budget of
        # a resident decode step - config 2 runs the whole model this way).
        ck = (key, ptr, mode)
        ref = self._refs.get(ck)
        if ref is None:
            shift = (self.pinfo[key].chunk_values.bit_length() - 1) if key in self.pinfo else 20
            n, k = self._unit_shape(key)
            ref = dgemm.WeightRef(ptr, 0, n, k, mode, shift)
            if len(self._refs) > 8192:
                self._refs.clear()
            self._refs[ck] = ref
        return ref

    def _done(self, lease) -> None:
        if isinstance(lease, tuple) and lease[0] == "native":  # release + run-ahead bound, natively
            self._us.release(lease[1], self._stream_handle(), not self.fake)
        elif isinstance(lease, tuple):  # a gather slot read by the kernels just enqueued
            self.gather.done(lease[1])
            self._mark_consumed()
        elif lease is not None:
            lease.release(0 if self.fake else None)
            self._mark_consumed()

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
        dv = self.dev
        # Deferred epilogues: the qkv GEMM's split-K sum runs in k_rope_kv (any
        # TP degree: QKV is column-parallel, nothing to reduce across ranks);
        # with one TP rank the o / down GEMMs' residual adds also run in the
        # next k_rmsnorm - 3 fewer launches per layer, bit-identical to the
        # separate reduce. Under TP the o / down outputs are partial sums that
        # must be all-reduced over the ranks before the residual add, so their
        # epilogue cannot run on the local split-K partials.
        fuse_qkv = self.fuse_epilogues
        fuse = self.fuse_epilogues and self.world == 1
        fuse_down = fuse and len(self.layout.roles["wd"]) == 1
        # GEMM inputs (h, a, g) in the MFMA fragment order (dgemm.to_frag): every
        # activation fragment is one contiguous 1 KB load in the GEMM
        xf = self.x_frag
        xr = self._xrows = B if xf else None
        pend = None  # the previous layer's deferred down projection
        for i in range(cfg.n_layers):
            h = fused.rms_norm(x, self.norm_w[2 * i], cfg.norm_eps, device_index=dv, pending=pend, out_frag=xf)
            pend = None
            lease, w = self._use(("layer", i, "wqkv"))
            qkv = dgemm.linear(h, w, device_index=dv, defer=fuse_qkv, x_rows=xr)
            self._done(lease)
            kvl = self._kv_layer(i, pos)
            q = self._rope_append(i, pos, kvl, qkv)
            a = fused.attention(q, kvl, pos + 1, device_index=dv, out_frag=xf)
            lease, w = self._use(("layer", i, "wo"))
            if fuse:
                o = dgemm.linear(a, w, device_index=dv, defer=True, x_rows=xr)
                self._done(lease)
                h = fused.rms_norm(x, self.norm_w[2 * i + 1], cfg.norm_eps, device_index=dv, pending=o,
                                   out_frag=xf)
            else:
                x = self._row_parallel(a, w, x)
                self._done(lease)
                h = fused.rms_norm(x, self.norm_w[2 * i + 1], cfg.norm_eps, device_index=dv, out_frag=xf)
            g = torch.empty(dgemm.frag_rows(B) if xf else B, self.f_local, dtype=torch.bfloat16, device=x.device)
            for name in self.layout.roles["wgu"]:
                r0, r1 = self.layout.rows[name]
                lease, w = self._use(("layer", i, name))
                if xf:
                    dgemm.linear(h, w, "silu_mul", out=g, out_frag=True, out_col0=r0, device_index=dv, x_rows=xr)
                else:
                    dgemm.linear(h, w, "silu_mul", out=g[:, r0:r1], device_index=dv)
                self._done(lease)
            if fuse_down:
                lease, w = self._use(("layer", i, self.layout.roles["wd"][0]))
                pend = dgemm.linear(g, w, device_index=dv, defer=True, x_rows=xr)
                self._done(lease)
            else:
                x = self._down(i, g, x)
        x = fused.rms_norm(x, self.final_norm, cfg.norm_eps, device_index=dv, pending=pend, out_frag=xf)
        logits = torch.empty(B, self.vocab_local, dtype=torch.bfloat16, device=x.device)
        for j, (r0, r1) in enumerate(self.head_rows):
            lease, w = self._use(("head", j))
            dgemm.linear(x, w, out=logits[:, r0:r1], device_index=dv, x_rows=xr)
            self._done(lease)
        if self.keep_logits:
            # tp: vocab shards of every sequence; shards: every rank's own sequences
            self.last_logits = comm.all_gather_cat(logits.float(), dim=0 if self.sworld > 1 else -1)
        nxt = tpmod.vocab_parallel_argmax(logits, self.rank, self.world)
        self.pos += 1
        return nxt

    def _row_parallel(self, a: torch.Tensor, w: "dgemm.WeightRef", x: torch.Tensor) -> torch.Tensor:
        """x + (a @ W^T) summed over TP ranks. One rank: the residual add is fused
        into the GEMM epilogue (in place on x); else partial GEMM + RCCL all-reduce."""
        if self.world == 1:
            return dgemm.linear(a, w, "resid", resid=x, out=x, device_index=self.dev, x_rows=self._xrows)
        o = dgemm.linear(a, w, device_index=self.dev, x_rows=self._xrows)
        return x + tpmod.row_parallel_reduce(o)

    def _down(self, i: int, g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        """x + g @ Wd^T over the down projection's row parts (and TP ranks). One
        rank: each part's residual add is fused into its GEMM epilogue, in place
        on x[:, n0:n1]; else the parts fill one partial sum for one all-reduce."""
        o = x if self.world == 1 else torch.empty_like(x)
        for name in self.layout.roles["wd"]:
            n0, n1 = self.layout.rows[name]
            lease, w = self._use(("layer", i, name))
            if self.world == 1:
                dgemm.linear(g, w, "resid", resid=x[:, n0:n1], out=x[:, n0:n1], device_index=self.dev,
                             x_rows=self._xrows)
            else:
                dgemm.linear(g, w, out=o[:, n0:n1], device_index=self.dev, x_rows=self._xrows)
            self._done(lease)
        return x if self.world == 1 else x + tpmod.row_parallel_reduce(o)

    def reset(self, position: Optional[int] = None) -> None:
        self.pos = self.ctx if position is None else position

    def close(self) -> None:
        if self.gather is not None:
            self.gather.drain()
            if getattr(self, "_gcache_lease", None) is not None:
                self._gcache_lease.release(0 if self.fake else None)
                lib.sync_all()
                self._gcache.free()
                self._gcache, self._gcache_lease = None, None
        self._us = None  # (its run-ahead events synchronised) before the ranges go
        self.kv_lease.release(0 if self.fake else None)
        for lease in self._pin_leases:
            lease.release(0 if self.fake else None)
        self._pin_leases, self._pinned, self._kv_pinned = [], {}, {}
        lib.sync_all()
        for b in [self.embed, self.kv] + list(self.ubuf.values()):
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
    norms = model.norm_w.float().cpu().to(dev)
    for i in range(cfg.n_layers):
        w = {n: model.host_matrix(("layer", i, n)).float().to(dev) for n in model.layout.roles}
        h = D.rms_norm(x, norms[2 * i], cfg.norm_eps)
        qkv = h @ w["wqkv"].t()
        q = qkv[:, :model.hq * hd].view(B, model.hq, hd)
        k = qkv[:, model.hq * hd:(model.hq + model.hkv) * hd].view(B, model.hkv, hd)
        v = qkv[:, (model.hq + model.hkv) * hd:].view(B, model.hkv, hd)
        q, k = D.apply_rope(q, cos, sin), D.apply_rope(k, cos, sin)
        kvh = model.host_kv(i).float().to(dev)
        kc = kvh[0].clone()
        vc = kvh[1].clone()
        kc[:, :, pos] = k
        vc[:, :, pos] = v
        a = D.gqa_decode_attention(q, kc, vc, pos + 1)
        x = x + a @ w["wo"].t()
        h = D.rms_norm(x, norms[2 * i + 1], cfg.norm_eps)
        x = x + D.silu_mul(h @ w["wgu"].t()) @ w["wd"].t()
    x = D.rms_norm(x, norms[2 * cfg.n_layers], cfg.norm_eps)
    head = model.host_matrix(("head",)).float().to(dev)
    return x @ head.t()


def smoke(device: int = 0) -> dict:
    """Tiny tiered decode on cuda:0 with the HBM budget below the footprint, on
    the headline bench's path (runtime-decided residency - planner off - with
    rANS-packed weights and KV), checked against the plain fp32 PyTorch
    reference (``reference_step``) every step: a wrong-logits regression in the
    default path fails here, not just a path that moves no bytes."""
    if not lib.is_initialized():
        rt.init("hip", host_budget_mb=4096)
    cfg = CONFIGS["small"]
    m = TieredLlama(cfg, batch=4, context=128, max_new_tokens=8, oversub=2.0, device=device, lookahead=1,
                    weight_format="ans", kv_format="ans", planner="off")
    m.keep_logits = True
    tok = torch.randint(0, cfg.vocab, (4,), device=m.tdev)
    max_err = 0.0
    for _ in range(3):
        ref = reference_step(cfg, m, tok.cpu(), m.pos).float()
        tok = m.step(tok)
        torch.cuda.synchronize()
        got = m.last_logits.float().to(ref.device)
        err = (got - ref).abs().max().item()
        max_err = max(max_err, err)
        assert torch.allclose(got, ref, atol=0.05, rtol=0.05), f"smoke logits off the fp32 reference: max err {err}"
        tok = ref.argmax(-1).to(m.tdev)  # stay on the reference's trajectory
    s = lib.stats()
    out = {"tokens": tok.tolist(), "max_logit_err_vs_fp32": round(max_err, 5), "evictions": s["evictions"],
           "bytes_htd": s["bytes_xfer_htd"], "plan": m.describe()}
    m.close()
    assert s["bytes_xfer_htd"] > 0, "smoke did not stream any weights"
    return out
