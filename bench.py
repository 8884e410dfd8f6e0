#!/usr/bin/env python3
"""Flagship benchmark: Llama-3-70B decode at 2x HBM oversubscription.

Metric (BASELINE.json): "tokens/sec Llama-3-70B 2x oversubscribe; HBM<->CXL GB/s
at 1/2/4/8 GPU". The reference publishes no number (published: {}), so
``vs_baseline`` is null.

Config: Llama-3-70B architecture, random-init bf16 weights (no checkpoints are
available offline), synthetic prefilled KV cache of ``--context`` tokens, greedy
decode of ``--batch`` sequences. Every weight and the KV cache are runtime-managed;
the per-GPU HBM arena is capped at (managed footprint / oversub), so half the
model lives in host DRAM and streams through the migration ring every step.
With N GPUs (one process per GPU, RCCL over xGMI; each process's runtime
manages only its own GPU and rests its host tier on that GPU's NUMA node) the
global batch is fixed (strong scaling) and ``--parallel`` picks how the model is
split:
  * ``tp`` (default): Megatron tensor parallelism - each rank streams only its
    1/N of every layer over its own PCIe link, 2 all-reduces per layer;
  * ``shards`` (config 4, peermem-style P2P shards): each rank owns 1/N of every
    unit (preferred on its GPU / streamed from its host DRAM), units are
    all-gathered over xGMI before use, each rank decodes B/N sequences.

One step = one decode token for every sequence (weights streamed, KV appended,
greedy sampling). ``value`` = global tokens/s = batch * K / max-over-ranks time.

Weights rest losslessly packed (rANS over the exponents, ~0.66x, bit-exact
bf16 after unpack) in every tier and are unpacked per matrix into a bf16 staging
buffer right before it is used (the KV prefix likewise, per layer); the
oversubscription ratio and HBM budget are computed on the logical bf16 footprint
(weights + KV + embedding + head), and the staging buffers are carved out of that
budget. Streamed matrices cross PCIe on the SDMA engines (the runtime's default
ring engine, copy_engine=3: ROCr hsa_amd_memory_async_copy_on_engine driven by
the ring worker), so no CU copy kernel competes with the compute kernels. ``--weights bf11`` (decoded
in the GEMM's registers) and ``--weights bf16`` run the other paths.

Also reported (aux): HBM<->host and HBM<->CXL GB/s measured through the runtime's
rings (the CXL pool is an emulated NUMA node when the box has no CXL device).

  python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
if hasattr(__import__("signal"), "pthread_sigmask"):
    # Hang dumps (ogkm.diag): SIGUSR1 is blocked before torch / HIP start any
    # thread, so every thread inherits the mask and only the dump thread takes it.
    import signal as _signal
    _signal.pthread_sigmask(_signal.SIG_BLOCK, {_signal.SIGUSR1})


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--context", type=int, default=1024)
    ap.add_argument("--oversub", type=float, default=2.0)
    ap.add_argument("--lookahead", type=int, default=int(os.environ.get("OGKM_LOOKAHEAD", "1")),
                    help="streamed tensors in flight beyond the one in use (each costs a staging slot of HBM)")
    ap.add_argument("--no-aux", action="store_true", help="skip the HBM<->host/CXL bandwidth probe")
    ap.add_argument("--weights", choices=("auto", "bf11", "bf12", "ans", "bf16"), default="auto",
                    help="bf11/ans/bf12: weights rest losslessly packed (~0.70x / ~0.67x / 0.75x) in every tier (HBM "
                         "included); bf11 is decoded in the GEMM's registers, ans/bf12 unpacked per matrix into a "
                         "bf16 staging buffer; bf16: raw weights")
    ap.add_argument("--no-packed", action="store_true",
                    help="with --weights bf16: raw host copies instead of BF12 copies decoded in the H2D kernel")
    ap.add_argument("--kv-format", choices=("auto", "bf11", "ans", "bf16"), default="auto",
                    help="bf11: the prefilled KV context rests losslessly packed in HBM (unpacked per layer into a "
                         "one-layer scratch), decode tokens raw; bf16: raw KV cache")
    ap.add_argument("--tiers", choices=("host", "host+cxl"), default="host",
                    help="where streamed weights rest: host DRAM, or interleaved host DRAM / CXL.mem (three-tier)")
    ap.add_argument("--cxl-frac", type=float, default=0.5, help="share of streamed tensors resting in CXL.mem")
    ap.add_argument("--simulate-tp", type=int, default=0,
                    help="single-process run of TP rank 0 of N (per-GPU shard of an N-GPU job; collectives "
                         "skipped, numerics not meaningful) - for configs larger than the box, e.g. 405B tp8")
    ap.add_argument("--parallel", choices=("tp", "shards"), default="tp",
                    help="multi-GPU split: tensor parallel, or peer-shard weights all-gathered over xGMI")
    ap.add_argument("--backend", choices=("hip", "fake"), default="hip",
                    help="fake: CPU-only runtime (fake GPUs, gloo) - rehearses the multi-rank path without a GPU")
    ap.add_argument("--fake-hbm-mb", type=int, default=1024)
    ap.add_argument("--dump-logits", default="",
                    help="write the last step's logits [global batch, vocab] (fp32) to this file (rank 0)")
    ap.add_argument("--planner", choices=("static", "off"), default="off",
                    help="off (default): no residency plan - every weight prefers HBM, nothing is pinned; the "
                         "runtime decides residency from the model's next-use hints (Belady order, spread "
                         "classes) and its prefetch / eviction. static: a hand-made plan pins whole layers")
    ap.add_argument("--kv-tiering", action="store_true",
                    help="KV prefixes as evictable per-layer units (resident with their layer, else streamed)")
    ap.add_argument("--allocator", action=argparse.BooleanOptionalAction, default=None,
                    help="route torch CUDA allocations through the runtime's HBM arena (pluggable allocator); "
                         "default: on for the HBM-resident single-GPU run (--oversub 1, config 2 - the allocator "
                         "baseline), off otherwise")
    ap.add_argument("--torch-managed", action="store_true",
                    help="run a stock torch.nn Llama (models/torch_llama.py) under ogkm.managed(): every tensor "
                         "oversubscribes HBM through the transparent mode, no hand-planned residency (1 GPU)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print the per-rank residency / traffic plan (JSON lines) of 70B and 405B, tp and shards, "
                         "at N = 1, 2, 4, 8 GPUs - host and CXL NUMA nodes, PCIe and xGMI GB/step, predicted "
                         "ms/step - without allocating anything (no GPU needed)")
    ap.add_argument("--same-gpu", action="store_true",
                    help="test drill: every rank runs on GPU 0 (own runtime and arena each) over a gloo process group "
                         "- RCCL refuses two ranks on one device; exercises the multi-rank kernels on a 1-GPU box")
    ap.add_argument("--launch-timeout", type=float, default=float(os.environ.get("OGKM_LAUNCH_TIMEOUT_S", "3000")),
                    help="--gpus N without torchrun: seconds the rank processes may run before all are killed")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _request_dumps(procs, wait_s: float = None) -> None:
    """SIGUSR1 to every still-running rank (ogkm.diag dumps its threads' stacks and
    the runtime's rings / leases to stderr), then give the dumps time to finish."""
    import signal

    if wait_s is None:
        wait_s = float(os.environ.get("OGKM_HANG_DUMP_WAIT_S", "8"))
    live = [p for p in procs if p.poll() is None]
    for p in live:
        try:
            os.kill(p.pid, signal.SIGUSR1)
        except ProcessLookupError:
            pass
    if live:
        time.sleep(wait_s)


def _kill_groups(procs, grace_s: float = 10.0) -> None:
    """SIGTERM every still-running rank's process group, SIGKILL what is left after ``grace_s``."""
    import signal

    live = [p for p in procs if p.poll() is None]
    for p in live:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
    t_end = time.monotonic() + grace_s
    for p in live:
        try:
            p.wait(timeout=max(0.1, t_end - time.monotonic()))
        except Exception:  # noqa: BLE001 - still alive: the hard kill below
            pass
    for p in live:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def launch_ranks(a) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N rank processes of this
    script (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, RCCL
    over xGMI - or gloo with ``--backend fake``) and wait for them.

    This process never touches the GPU (torch is not even imported), so no
    GPU-initialised process is ever replaced or forked. Every rank runs in its
    own process group; if one exits non-zero, or the job outlives
    ``--launch-timeout``, every other rank is killed (SIGTERM, then SIGKILL)
    and the launcher exits non-zero. Rank 0's stdout (the JSON line) is
    inherited, so it reaches our stdout unchanged. Returns the exit code."""
    import subprocess

    n = a.gpus
    port = _free_port()
    base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(port), OGKM_BENCH_LAUNCHED="1")
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    try:
        for r in range(n):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0", ROLE_RANK=str(r))
            procs.append(subprocess.Popen(cmd, env=env, start_new_session=True,
                                          stdout=None if r == 0 else subprocess.DEVNULL))
        deadline = time.monotonic() + a.launch_timeout
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"[bench] rank {r} exited with status {c}: stopping the other ranks", file=sys.stderr,
                      flush=True)
                _kill_groups(procs)
                return c if c > 0 else 1
            if all(c == 0 for c in codes):
                return 0
            if time.monotonic() > deadline:
                print(f"[bench] ranks still running after {a.launch_timeout:.0f} s: dumping their stacks, "
                      f"then killing all {n}", file=sys.stderr, flush=True)
                _request_dumps(procs)
                _kill_groups(procs)
                return 124
            time.sleep(0.2)
    except BaseException:
        _kill_groups(procs)
        raise


HBM_USABLE_GB = 270.0  # of the 288 GB per MI355X (runtime / RCCL / activation reserve)


def plan_only(a) -> None:
    """Dry-run residency plans (models/llama.py TieredLlama(dry_run=True) +
    traffic()): what every rank of an N-GPU job would hold, stream and
    exchange per decode step, before any multi-GPU run is launched."""
    from ogkm.models import llama
    try:
        from ogkm._native import lib
        n_dev = lib.device_count() if lib.is_initialized() else 0
    except Exception:  # noqa: BLE001
        n_dev = 0
    models = [a.model] if a.model not in ("llama3-70b",) else ["llama3-70b", "llama3-405b"]
    for model in models:
        cfg = llama.CONFIGS[model]
        tiers = "host+cxl" if model == "llama3-405b" else a.tiers
        for parallel in ("tp", "shards"):
            for n in (1, 2, 4, 8):
                if parallel == "shards" and n == 1:
                    continue
                wf = "ans" if a.weights == "auto" else a.weights
                kf = "ans" if a.kv_format == "auto" else a.kv_format
                kw = dict(batch=a.batch, context=a.context, max_new_tokens=a.warmup + a.steps + 3, tp_rank=0,
                          tp_world=n, weight_format=wf, kv_format=kf, parallel=parallel, tiers=tiers,
                          cxl_frac=a.cxl_frac, dry_run=True)
                m = llama.TieredLlama(cfg, oversub=a.oversub, **kw)
                oversub = a.oversub
                if m.budget / 1e9 > HBM_USABLE_GB:  # the logical ratio does not fit one MI355X: cap at its HBM
                    oversub = m.footprint / (HBM_USABLE_GB * 1e9)
                    m = llama.TieredLlama(cfg, oversub=oversub, **kw)
                d, t = m.describe(), m.traffic()
                # one process per GPU: GPUs 0-3 sit on socket 0, 4-7 on socket 1 (MI355X 8-GPU node);
                # each rank's host tier and its nearest (emulated) CXL pool are on its GPU's socket
                nodes = [(lib.device_numa_node(r) if r < n_dev else r // 4) for r in range(n)]
                out = {"plan": model, "parallel": f"{parallel}{n}", "n_gpus": n, "oversubscription": round(oversub, 3),
                       "global_batch": a.batch, "seq_len": a.context, "weight_format": wf, "kv_format": kf,
                       "tiers": tiers,
                       "per_rank": {"host_numa_node": nodes, "cxl_numa_node": nodes,
                                    "footprint_gb": round(d["footprint_gb"], 2), "hbm_budget_gb": round(d["hbm_budget_gb"], 2),
                                    "resident_layers": d["resident_layers"], "streamed_layers": d["streamed_layers"],
                                    "pcie_gb_per_step": round(t["pcie_gb"], 3),
                                    "cxl_gb_per_step": round(d["cxl_streamed_gb_per_step"], 3),
                                    "xgmi_gb_per_step": round(t["xgmi_gb"], 3), "hbm_gb_per_step": round(t["hbm_gb"], 2),
                                    "collectives_per_step": t["collectives"],
                                    "pcie_ms": round(t["pcie_ms"], 2), "xgmi_ms": round(t["xgmi_ms"], 2),
                                    "hbm_ms": round(t["hbm_ms"], 2)},
                       "predicted_ms_per_step": round(t["predicted_ms"], 2),
                       "predicted_tokens_per_s": round(a.batch / (t["predicted_ms"] / 1e3), 1),
                       "model": "PCIe %.1f GB/s, HBM %.0f GB/s, xGMI %.0f GB/s per link, %.0f us per collective"
                                % (llama.PLAN_PCIE_GBPS, llama.PLAN_HBM_GBPS, __import__("ogkm.parallel.topology",
                                   fromlist=["x"]).XGMI_LINK_GBPS, __import__("ogkm.parallel.topology",
                                   fromlist=["x"]).COLLECTIVE_LATENCY_US)}
                print(json.dumps(out), flush=True)


def run_torch_managed(a) -> None:
    """Stock torch model under the transparent managed mode: parameters and KV
    cache are torch tensors allocated through the runtime's pluggable allocator;
    the HBM arena is capped at footprint / oversub, and every aten op holds the
    managed tensors it touches (open-gpu-kernel-modules_amd/managed.py)."""
    import torch

    import ogkm
    from ogkm import allocator, rt
    from ogkm._native import lib
    from ogkm.models import llama, torch_llama

    cfg = llama.CONFIGS[a.model]
    foot = torch_llama.footprint_bytes(cfg, a.batch, a.context)
    budget = int(foot / a.oversub)
    # allocations >= OGKM_MANAGED_MIN_MB are managed (evictable) ranges; the
    # op-trace prefetcher looks OGKM_MANAGED_LOOKAHEAD_MB ahead (-1: a quarter of the arena)
    allocator.enable(managed_min_mb=int(os.environ.get("OGKM_MANAGED_MIN_MB", "1")))
    # packed host copies (packer.cpp): weights dropped clean from HBM are
    # ANS1-packed by host encoder threads during warmup; OGKM_PACK=0 keeps raw
    pack = int(os.environ.get("OGKM_PACK", "1"))
    rt.init("hip", hbm_budget={0: budget}, host_budget_mb=0, pack_host_copies=pack,
            pack_threads=int(os.environ.get("OGKM_PACK_THREADS", "12")))
    torch.cuda.set_device(0)
    prefill = a.context - (a.warmup + a.steps) - 1
    la = int(os.environ.get("OGKM_MANAGED_LOOKAHEAD_MB", "-1"))
    mode = ogkm.managed(lookahead_bytes=None if la < 0 else la << 20)
    t_init = time.perf_counter()
    with mode:
        model = torch_llama.build_on_device(cfg, a.batch, a.context, "cuda", seed=1234, prefill=prefill)
        # Harness-side advice (no framework call inside the model): weights are
        # only read by decode, so their host copies stay valid while resident
        # and evicting them costs no copy-out.
        for p in model.parameters():
            if allocator.is_managed(p):
                allocator.set_read_mostly(p)
        g = torch.Generator(device="cpu").manual_seed(42)
        tok = torch.randint(0, cfg.vocab, (a.batch,), generator=g).to("cuda")
        pos = prefill
        torch.cuda.synchronize()
        init_s = time.perf_counter() - t_init
        for _ in range(a.warmup):
            tok = model.step(tok, pos)
            pos += 1
        torch.cuda.synchronize()
        # setup, not timed: let the packer finish the host copies the warmup
        # steps released (then one more step refills HBM from them)
        t_p = time.perf_counter()
        packed_all = True
        if pack:
            limit = float(os.environ.get("OGKM_PACK_WAIT_S", "900"))
            while not lib.pack_wait(20000):  # progress lines: a silent minute reads as a hang
                ps = lib.pack_stats()
                print(f"packing: {ps['packed_blocks']} blocks packed, {ps['queued']} queued "
                      f"({time.perf_counter() - t_p:.0f} s)", file=sys.stderr, flush=True)
                if time.perf_counter() - t_p > limit:
                    packed_all = False
                    break
        pack_s = time.perf_counter() - t_p
        if pack:
            tok = model.step(tok, pos)
            pos += 1
            torch.cuda.synchronize()
        lib.reset_counters()
        al0 = allocator.stats()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tok = model.step(tok, pos)
            pos += 1
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        al1 = allocator.stats()
    s = lib.stats()
    census = _block_census() if os.environ.get("OGKM_TM_CENSUS") == "1" else None
    name = {"llama3-70b": "Llama-3-70B", "llama3-405b": "Llama-3-405B", "llama3-8b": "Llama-3-8B"}.get(a.model, a.model)
    out = {
        "metric": f"tokens/sec {name} {a.oversub:g}x oversubscribe (stock torch model, transparent managed mode)",
        "value": round(a.batch * a.steps / dt, 3),
        "unit": "tokens/s",
        "n_gpus": 1,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random-init weights, synthetic prefilled KV cache)",
        "config": {"model": a.model, "global_batch": a.batch, "seq_len": a.context, "parallelism": "tp1",
                   "engine": "torch.nn + ogkm.managed()", "footprint_gb": round(foot / 1e9, 2),
                   "hbm_budget_gb": round(budget / 1e9, 2), "oversubscription": round(foot / budget, 3)},
        "aux": {"htd_gb_per_step": round(s["bytes_xfer_htd"] / a.steps / 1e9, 2),
                "dth_gb_per_step": round(s["bytes_xfer_dth"] / a.steps / 1e9, 2),
                "link_gbps": round(s["bytes_xfer_htd"] / dt / 1e9, 2), "evictions": s["evictions"],
                "vmm_remaps": s["vmm_remaps"], "tlb_flushes": s["tlb_flushes"], "ops": mode.ops,
                "host_ms_per_step": {k: round(s[k + "_ns"] / 1e6 / a.steps, 1)
                                     for k in ("place_stable", "vmm_map", "vmm_unmap", "tlb_flush", "stable_wait")},
                "ring_per_step": _ring_per_step(s, a.steps),
                "faulted_ops": mode.faulted_ops, "prefetches": mode.prefetches, "init_s": round(init_s, 1),
                "pack": dict(lib.pack_stats(), wait_s=round(pack_s, 1), drained=packed_all,
                             decodes_per_step=s["packed_decodes"] // max(1, a.steps),
                             expansions=s["pack_expansions"],
                             seg_decodes_per_step=s["seg_decodes"] // max(1, a.steps),
                             seg_expansions=s["seg_expansions"]),
                "trace_len": len(mode._trace), "hinted_ops": mode.hinted_ops, "trace_misses": mode.trace_misses,
                "allocs_per_step": (al1["allocs"] - al0["allocs"]) // max(1, a.steps), "alloc_peak_gb":
                round(al1["peak"] / 1e9, 2), "managed_min_mb": int(os.environ.get("OGKM_MANAGED_MIN_MB", "1")),
                "lookahead_mb": la, "block_census": census,
                "spread": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in lib.spread_stats(0).items()}},
    }
    print(json.dumps(out), flush=True)


def _block_census(top: int = 8) -> dict:
    """Where every managed 2 MB block rests (diagnostic, after the timed steps):
    HBM-resident or not, host copy packed / raw; the ranges with the most
    non-resident raw blocks (what refills move unpacked)."""
    from collections import Counter

    from ogkm._native import lib
    kinds, per_range = Counter(), []
    for rid in lib.range_ids():
        info = lib.range_info(rid)
        raw_out = 0
        for bi in range(info["nblocks"]):
            try:
                ri = lib.residency_info(rid, bi << 21)
            except Exception:  # noqa: BLE001 - a range freed meanwhile
                break
            tiers = [e["tier"] for e in ri["resident_on"]]
            packed = any(e.get("encoded_bytes") for e in ri["resident_on"] if e["tier"] != "gpu")
            seg = any(e.get("packed_segments") for e in ri["resident_on"] if e["tier"] != "gpu")
            gpu = "gpu" in tiers
            host = any(t != "gpu" for t in tiers)
            key = ("gpu" if gpu else "nogpu") + ("+segpacked" if seg else "+packed" if packed else "+raw" if host else "")
            kinds[key] += 1
            raw_out += (not gpu) and host and not packed
        if raw_out:
            per_range.append((raw_out, info["name"], info["size"]))
    per_range.sort(reverse=True)
    return {"blocks": dict(kinds), "raw_not_resident_top": [
        {"blocks": n, "name": nm, "mb": round(sz / 2**20, 1)} for n, nm, sz in per_range[:top]]}


def _ring_per_step(s: dict, steps: int) -> dict:
    """DMA ring workers (all rings summed): ms per step waiting for copy
    dependencies, in engine copies, idle; engine copy calls per step."""
    out = {k: round(s.get(f"ring_{k}_ns", 0) / 1e6 / max(1, steps), 1) for k in ("fence_wait", "copy", "idle")}
    out["copy_calls"] = s.get("ring_copy_calls", 0) // max(1, steps)
    for k in ("packed_decodes", "ring_merged_batches", "decode_reuse_waits", "victim_risen_seen"):
        if s.get(k):
            out[k] = s[k] // max(1, steps)
    if s.get("victim_search_ns"):  # host time in next-use victim searches
        out["victim_search_ms"] = round(s["victim_search_ns"] / 1e6 / max(1, steps), 1)
    return out


PROBE_KEYS = ("host_to_hbm", "hbm_to_host", "cxl_to_hbm", "hbm_to_cxl")


def bandwidth_probe(dev: int, barrier, nbytes: int = 1 << 30) -> tuple[dict, dict]:
    """HBM<->host and HBM<->CXL GB/s through the runtime's migration rings
    (``lib.ring_copy``: the ring's configured engine, SDMA by default). Every
    rank runs it at once (``barrier`` before each timed direction),
    so with N GPUs the sum over ranks is the node's aggregate HBM<->host/CXL rate
    (BASELINE metric: "HBM<->CXL GB/s at 1/2/4/8 GPU"). Returns (rates, info)."""
    import torch

    from ogkm import cxl
    from ogkm._native import lib

    out = {}
    g = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{dev}")
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    for name, ring, dst, src in (("host_to_hbm", 0, g.data_ptr(), h.data_ptr()),
                                 ("hbm_to_host", 1, h.data_ptr(), g.data_ptr())):
        lib.ring_copy(dev, ring, dst, src, nbytes, True)
        barrier()
        t0 = time.perf_counter()
        for _ in range(3):
            lib.ring_copy(dev, ring, dst, src, nbytes, True)
        out[name] = 3 * nbytes / (time.perf_counter() - t0) / 1e9
    del g, h
    info = cxl.get_info()
    near = lib.cxl_nearest_node(lib.host_node()) if info["numa_nodes"] else lib.host_node()
    far = [n for n in info["numa_nodes"] if n != near]
    meta = {"cxl_numa_node": near, "host_numa_node": lib.host_node(),
            "emulated": bool(info["emulated"] or not info["numa_nodes"])}
    try:
        # the rank's own pool (nearest) is what tiering uses; the other socket's
        # pool is measured too (remote CXL: the same full-rate SDMA engines)
        r = cxl.measure_bandwidth(dev, nbytes, iters=3, node=near, barrier=barrier)
        out["cxl_to_hbm"], out["hbm_to_cxl"] = r["cxl_to_gpu_gbps"], r["gpu_to_cxl_gbps"]
        if far:
            r2 = cxl.measure_bandwidth(dev, nbytes, iters=3, node=far[0], barrier=barrier)
            meta["remote"] = {"cxl_numa_node": far[0], "cxl_to_hbm": round(r2["cxl_to_gpu_gbps"], 2),
                              "hbm_to_cxl": round(r2["gpu_to_cxl_gbps"], 2)}
    except Exception as e:  # no CXL / registration refused: report, do not fail the bench
        out["cxl_to_hbm"] = out["hbm_to_cxl"] = 0.0
        meta["error"] = str(e)
    return out, meta


def probe_all_ranks(dev: int, rank: int) -> dict:
    """Run the probe on every rank concurrently; rank 0 gets per-GPU and aggregate GB/s."""
    import torch

    from ogkm.parallel import comm

    rates, meta = bandwidth_probe(dev, comm.barrier)
    e = comm.env()
    t = torch.tensor([[rates[k] for k in PROBE_KEYS]], dtype=torch.float64,
                     device=f"cuda:{dev}" if e.backend == "nccl" else "cpu")
    allr = comm.all_gather_cat(t, dim=0).cpu()  # [world, 4]
    return {
        "host_to_hbm_gbps": round(rates["host_to_hbm"], 2),
        "hbm_to_host_gbps": round(rates["hbm_to_host"], 2),
        "hbm_cxl_gbps": {"cxl_to_hbm": round(rates["cxl_to_hbm"], 2), "hbm_to_cxl": round(rates["hbm_to_cxl"], 2),
                         **meta},
        # all N GPUs copying at once (each over its own PCIe link to the host / CXL pool)
        "aggregate_gbps": {"n_gpus": int(allr.shape[0]),
                           **{k: round(float(allr[:, j].sum()), 2) for j, k in enumerate(PROBE_KEYS)},
                           "min_per_gpu": {k: round(float(allr[:, j].min()), 2) for j, k in enumerate(PROBE_KEYS)}},
    }


def main() -> None:
    a = parse()
    if a.plan_only:
        plan_only(a)
        return
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and a.gpus > 1:
        # no launcher: become one (before anything touches the GPU)
        if a.torch_managed or a.simulate_tp:
            raise SystemExit("--torch-managed / --simulate-tp are one-process runs: use --gpus 1")
        sys.exit(launch_ranks(a))
    if ws is not None and int(ws) != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={ws}: one rank process per GPU is required")
    if a.torch_managed:
        run_torch_managed(a)
        return
    # auto: packed (rANS) resting formats when part of the model streams - every
    # byte saved is a byte off PCIe; raw bf16 when everything is HBM-resident
    # (oversub <= 1), where packing would only add unpack work (8B: 2902 vs 925 tok/s).
    if a.weights == "auto":
        a.weights = "ans" if a.oversub > 1.0 else "bf16"
    if a.kv_format == "auto":
        a.kv_format = "ans" if a.oversub > 1.0 else "bf16"
    import torch

    from ogkm import rt
    from ogkm._native import lib
    from ogkm.models import llama
    from ogkm.parallel import comm

    fake = a.backend == "fake"
    if a.allocator is None:
        a.allocator = a.oversub == 1.0 and not a.torch_managed and a.gpus <= 1
    if a.allocator and not fake:
        # config 2: torch tensors share the runtime's HBM arena. Swapped in
        # before torch initialises its caching allocator (and before any CUDA
        # tensor exists); allocations resolve once the runtime is up.
        from ogkm import allocator
        allocator.enable()
    from ogkm import diag
    diag.install(tag=f"rank {os.environ.get('RANK', '0')} ")
    # torchrun does not signal a hung rank: each rank dumps itself if init or the
    # timed steps overrun (generous: a 405B init takes minutes)
    diag.arm(float(os.environ.get("OGKM_INIT_WATCHDOG_S", "1500")), "init")
    e = comm.init("gloo" if fake or a.same_gpu else None)
    if e.world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but the process group has {e.world} ranks")
    # failure drills for the launcher tests: one rank dies / hangs after joining the group
    if os.environ.get("OGKM_BENCH_FAIL_RANK", "") == str(e.rank):
        print(f"[bench] rank {e.rank}: injected failure", file=sys.stderr, flush=True)
        os._exit(3)
    hang_here = os.environ.get("OGKM_BENCH_HANG_RANK", "") == str(e.rank)
    if hang_here and os.environ.get("OGKM_BENCH_HANG_AT", "init") == "init":
        time.sleep(1e6)
    pg_world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    dev = 0 if a.same_gpu else e.local_rank
    if not fake:
        torch.cuda.set_device(dev)
    world = e.world
    cfg = llama.CONFIGS[a.model]
    # One process per GPU: this runtime manages only its own GPU (rings, fault
    # buffer and HBM arena on no other device), and its host tier sits on that
    # GPU's NUMA node.
    if fake:
        rt.init("fake", fake_devices=max(world, 1), fake_hbm_mb=a.fake_hbm_mb, host_budget_mb=4096,
                local_devices=1 << dev, fake_numa_nodes=2 if world > 1 else 1)
        a.no_aux = True
    else:
        rt.init("hip", host_budget_mb=0, local_devices=1 << dev)
    # No CXL hardware on the box: every NUMA node emulates a CXL pool, and each
    # rank demotes to the pool nearest its GPU's node (SLIT distance,
    # CxlTopology::nearest_node) - one pool per socket, as on a CXL-populated node.
    # The rank's own host node is left out of the emulated pool whenever another
    # node exists: a "CXL" tier on the host tier's node would be the same DRAM
    # counted twice, so the emulated pool is the other socket's memory (a farther
    # tier, reached over the socket link as a CXL expander on that socket would be).
    nodes = sorted({int(p.name[4:]) for p in Path("/sys/devices/system/node").glob("node[0-9]*")})
    cxl_kind = "cxl-device"
    if not lib.cxl_info()["numa_nodes"] and nodes:
        pool = [n for n in nodes if n != lib.host_node()] or nodes
        cxl_kind = ("emulated: other-socket DRAM" if pool != nodes
                    else "emulated: host-node DRAM (single NUMA node)")
        lib.cxl_rediscover(-1, "/sys", sum(1 << n for n in pool))
    aux = {}
    if not a.no_aux:
        aux = probe_all_ranks(dev, e.rank)
    comm.barrier()
    t_init = time.perf_counter()
    sim = a.simulate_tp > 1 and world == 1
    planner = a.planner
    model = llama.TieredLlama(cfg, batch=a.batch, context=a.context, max_new_tokens=a.warmup + a.steps + 3,
                              oversub=a.oversub, device=dev, tp_rank=e.rank, tp_world=a.simulate_tp if sim else world,
                              seed=1234, lookahead=a.lookahead, verbose=a.verbose, packed=not a.no_packed,
                              weight_format=a.weights, tiers=a.tiers, cxl_frac=a.cxl_frac, kv_format=a.kv_format,
                              parallel=a.parallel, planner=planner, kv_tiering=a.kv_tiering)
    plan = model.describe()
    init_s = time.perf_counter() - t_init
    g = torch.Generator(device="cpu").manual_seed(42)
    tok = torch.randint(0, cfg.vocab, (a.batch,), generator=g)
    tok = tok[model.b0:model.b0 + model.B]  # shards: this rank's sequences (tp: all of them)
    if not fake:
        tok = tok.to(f"cuda:{dev}")
    if a.dump_logits:
        model.keep_logits = True

    def sync():
        if not fake:
            torch.cuda.synchronize()
    diag.arm(float(os.environ.get("OGKM_STEP_WATCHDOG_S", str(120 + 30 * (a.warmup + a.steps)))), "decode steps")
    for w in range(a.warmup):
        if hang_here and w == 1:  # the drill's hang inside decode (runtime up, rings live)
            time.sleep(1e6)
        tok = model.step(tok)
    lib.reset_counters()
    comm.reset_stats()
    model.reset_stream_stats()
    model.diag = a.verbose
    if a.verbose:
        model.byte_trace = {}
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tok = model.step(tok)
    sync()
    comm.barrier()
    dt = comm.max_over_ranks(time.perf_counter() - t0)
    diag.disarm()
    s = lib.stats()
    xgmi_in = comm.STATS["allreduce_bytes_in"] + comm.STATS["allgather_bytes_in"]
    traffic = model.traffic()
    host_nodes = comm.all_gather_objects(lib.host_node())
    if a.dump_logits and e.rank == 0:
        torch.save(model.last_logits.float().cpu(), a.dump_logits)
    if a.verbose:
        # host enqueue time of one step (no sync inside) vs its synchronized time
        sync()
        h0 = time.perf_counter()
        tok = model.step(tok)
        h1 = time.perf_counter()
        sync()
        h2 = time.perf_counter()
        if e.rank == 0:
            print(f"[ogkm] one step: host enqueue {1e3 * (h1 - h0):.1f} ms, synchronized {1e3 * (h2 - h0):.1f} ms",
                  flush=True)
    if a.verbose and model.byte_trace is not None and e.rank == 0:
        res = {k: v for k, v in model.byte_trace.items() if model._is_resident(k) and v}
        print("[ogkm] H2D bytes/step around resident tensors:",
              {f"{k[0]}{k[1]}": round(v / a.steps / 1e9, 3) for k, v in res.items()}, flush=True)
        print(f"[ogkm] H2D GB/step total {s['bytes_xfer_htd'] / a.steps / 1e9:.2f}, planned streamed "
              f"{plan['streamed_gb_per_step']:.2f}", flush=True)
    tokens = a.batch * a.steps
    value = tokens / dt
    if e.rank == 0:
        name = {"llama3-70b": "Llama-3-70B", "llama3-405b": "Llama-3-405B", "llama3-8b": "Llama-3-8B"}.get(a.model,
                                                                                                        a.model)
        # the residency policy is config.planner ("off" = runtime-decided, the default)
        metric = f"tokens/sec {name} {a.oversub:g}x oversubscribe"
        if sim:  # one shard of an N-GPU job on one GPU: an upper bound, not a measured N-GPU rate
            metric += f" (tp{a.simulate_tp} rank-0 shard simulated on 1 GPU, collectives skipped)"
        out = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random-init weights, synthetic prefilled KV cache)",
            "config": {
                "model": a.model,
                "global_batch": a.batch,
                "seq_len": a.context,
                "parallelism": (f"tp{a.simulate_tp}-rank0-simulated" if sim
                                else f"{'shards' if a.parallel == 'shards' else 'tp'}{world}"),
                "backend": a.backend,
                # ranks in the process group that ran the step (RCCL on GPUs, gloo with --backend fake)
                "rccl_world": pg_world,
                "process_group": e.backend,
                "launcher": ("bench.py" if os.environ.get("OGKM_BENCH_LAUNCHED") == "1"
                             else "external" if world > 1 else "none"),
                "planner": model.planner,
                "gather_cache_gb_per_gpu": round(getattr(model, "gather_cache_bytes", 0) / 1e9, 3),
                "kv_tiering": a.kv_tiering,
                "torch_allocator": "ogkm-arena" if a.allocator else "torch-caching",
                "rank_host_numa_nodes": host_nodes,
                "tiers": plan["tiers"],
                "cxl_tier": cxl_kind,
                "kv_format": plan["kv_format"],
                "kv_resident_gb_per_gpu": round(plan["kv_resident_gb"], 2),
                "cxl_streamed_gb_per_step_per_gpu": round(plan["cxl_streamed_gb_per_step"], 2),
                "oversubscription": round(plan["oversubscription"], 3),
                # resting (packed) bytes of every managed range / HBM budget: the
                # physical oversubscription, vs the logical bf16 one above
                "physical_oversubscription": round(plan["physical_oversubscription"], 3),
                "hbm_budget_gb_per_gpu": round(plan["hbm_budget_gb"], 2),
                "managed_footprint_gb_per_gpu": round(plan["footprint_gb"], 2),
                "resident_layers": plan["resident_layers"],
                "streamed_layers": plan["streamed_layers"],
                "extra_resident_units": plan["extra_resident_units"],
                # measured host/CXL -> HBM bytes per step (planner off: what the runtime's
                # residency streamed); the static plan's estimate is labelled as such
                "streamed_gb_per_step_per_gpu": round((s["bytes_xfer_htd"] + s["bytes_xfer_ctd"]) / a.steps / 1e9, 2),
                "static_plan_streamed_gb_per_step_per_gpu": round(plan["streamed_gb_per_step"], 2),
                "weight_format": plan["weight_format"],
                "host_copy_format": (f"{plan['weight_format']}-lossless" if plan["weight_format"] != "bf16"
                                     else "bf12-lossless" if plan["packed_host_copies"] else "bf16"),
                "hbm_copy_format": ("bf11-lossless (decoded in the GEMM's registers)" if plan["weight_format"] == "bf11"
                                    else f"{plan['weight_format']}-lossless (unpacked per matrix)"
                                    if plan["weight_format"] in ("bf12", "ans") else "bf16"),
                "resting_bytes_ratio": round(plan["resting_layer_gb"] / plan["layer_gb"], 4),
            },
            "aux": {
                **aux,
                "link_gbps_per_gpu": round((s["bytes_xfer_htd"] + s["bytes_xfer_ctd"]) / max(dt, 1e-9) / 1e9, 2),
                # rank 0's per-step traffic: measured vs the plan (bench.py --plan-only prints the plan alone)
                "traffic_per_step_gb": {
                    "pcie_measured": round((s["bytes_xfer_htd"] + s["bytes_xfer_ctd"]) / a.steps / 1e9, 4),
                    "pcie_planned": round(traffic["pcie_gb"], 4),
                    "xgmi_measured": round(xgmi_in / a.steps / 1e9, 6),
                    "xgmi_planned": round(traffic["xgmi_gb"], 6),
                    "predicted_ms": round(traffic["predicted_ms"], 2)},
                "cxl_to_hbm_gbps_per_gpu": round(s["bytes_xfer_ctd"] / max(dt, 1e-9) / 1e9, 2),
                "evictions": s["evictions"],
                "ring_per_step": _ring_per_step(s, a.steps),
                "stream_stats_per_step": {k: round(v / a.steps, 1) for k, v in model.stream_stats().items()},
                # the runtime's keep / stream classes (planner off; csrc/core/spread.cpp)
                "spread": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in lib.spread_stats(dev).items()},
                "init_s": round(init_s, 1),
            },
        }
        print(json.dumps(out), flush=True)
    model.close()
    comm.shutdown()
    lib.shutdown()


if __name__ == "__main__":
    main()
