#!/usr/bin/env python3
"""Per-step diagnostics of the first decode steps after load: wall time and the
runtime's transfer / eviction counter deltas per step (finds start-up transients).

    python tools/diag_transient.py --model llama3-405b --simulate-tp 8 --tiers host+cxl --steps 5
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

KEYS = ("bytes_xfer_htd", "bytes_xfer_dth", "bytes_xfer_ctd", "bytes_xfer_dtc", "evictions", "evicted_bytes",
        "thrashing_detected", "revocations", "alloc_retries", "gpu_page_faults")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--simulate-tp", type=int, default=1)
    ap.add_argument("--tiers", default="host")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--weights", default="ans")
    ap.add_argument("--verify", action="store_true", help="checksum every unpacked unit against its host copy")
    ap.add_argument("--kv-format", default="ans")
    ap.add_argument("--dump-every", type=float, default=0.0,
                    help="dump every thread's Python stack every N s while a step runs (finds where a stall waits)")
    ap.add_argument("--dump-file", default="gpurun_out/stall_stacks.txt")
    ap.add_argument("--max-ratio", type=float, default=1.5,
                    help="fail when an early step takes more than this times the steady (last) step")
    a = ap.parse_args()
    import faulthandler
    import gc

    gc_t = {}

    def gc_cb(phase, info):  # a long cyclic-GC pause (finalizers) would show up here
        if phase == "start":
            gc_t["t"] = time.perf_counter()
        else:
            dt = time.perf_counter() - gc_t.get("t", time.perf_counter())
            if dt > 0.01:
                print(f"  gc gen{info['generation']} took {dt * 1e3:.1f} ms", flush=True)
    gc.callbacks.append(gc_cb)
    import importlib

    import torch
    importlib.import_module("open-gpu-kernel-modules_amd")
    from ogkm import rt
    from ogkm._native import lib
    from ogkm.models import llama

    rt.init("hip", host_budget_mb=0)
    # the emulated CXL pool, as bench.py: the NUMA node that is not the GPU's
    gpu_node = lib.device_numa_node(0)
    nodes = sorted({int(p.name[4:]) for p in Path("/sys/devices/system/node").glob("node[0-9]*")})
    other = [n for n in nodes if n != gpu_node]
    if not lib.cxl_info()["numa_nodes"] and other:
        lib.cxl_rediscover(other[0], "/sys")
    cfg = llama.CONFIGS[a.model]
    m = llama.TieredLlama(cfg, batch=64, context=1024, max_new_tokens=a.steps + 3, oversub=2.0, device=0,
                          tp_rank=0, tp_world=a.simulate_tp, seed=1234, lookahead=1, weight_format=a.weights,
                          tiers=a.tiers, kv_format=a.kv_format)
    tok = torch.randint(0, cfg.vocab, (64,)).cuda()
    unstaged = {}  # packed stream address -> unit (this step)
    orig_unstage = m._unstage
    ref_sum, seen = {}, []
    if a.verify:
        # checksum of every unit's packed stream as stored on the host
        for key in m.order:
            n = m.pinfo[key].nbytes // 4 * 4
            ref_sum[key] = int(m._buf(key).read(nbytes=n).view(torch.int32).sum(dtype=torch.int64))
        print(f"reference checksums of {len(ref_sum)} units", flush=True)

    def unstage(key, ptr):
        unstaged[ptr] = key
        if a.verify:  # checksum of what the unpack is about to read, in stream order (no host sync)
            n = m.pinfo[key].nbytes // 4 * 4
            v = rt._tensor_from_ptr(ptr, (n // 4,), torch.int32, "cuda", 0)
            seen.append((key, ptr, v.sum(dtype=torch.int64)))
        return orig_unstage(key, ptr)
    m._unstage = unstage
    times = []
    for i in range(a.steps):
        s0 = lib.stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if a.dump_every > 0:
            dump = open(a.dump_file, "a")
            dump.write(f"==== step {i}\n")
            dump.flush()
            faulthandler.dump_traceback_later(a.dump_every, repeat=True, file=dump)
        m.use_trace = []
        unstaged.clear()
        tok = m.step(tok)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if a.dump_every > 0:
            faulthandler.cancel_dump_traceback_later()
            dump.close()
        print(f"step {i}: host enqueue {t_enq * 1e3:.1f} ms", flush=True)
        slow = sorted(m.use_trace, key=lambda u: -(u[1] + u[2]))[:8]
        print("  slowest uses (key, acquire ms, wait ms):",
              [(u[0], round(u[1] * 1e3, 1), round(u[2] * 1e3, 1)) for u in slow], flush=True)
        s1 = lib.stats()
        d = {k: s1[k] - s0[k] for k in KEYS if k in s1}
        gb = {k: round(v / 1e9, 2) if "bytes" in k else v for k, v in d.items()}
        print(f"step {i}: {dt * 1e3:.1f} ms {gb}", flush=True)
        times.append(dt)
        if a.verify:
            bad = [(k, p, int(t)) for k, p, t in seen if int(t) != ref_sum[k]]
            print(f"  verify: {len(seen)} unpacks, {len(bad)} saw wrong packed bytes", flush=True)
            for k, p, t in bad[:6]:
                n = m.pinfo[k].nbytes // 4 * 4
                now = int(rt._tensor_from_ptr(p, (n // 4,), torch.int32, "cuda", 0).sum(dtype=torch.int64))
                res = [m._buf(k).residency(o) for o in range(0, m._buf(k).size, 2 << 20)]
                gpu_pages = [sum(r["pages"] for r in x["resident_on"] if r["tier"] == "gpu") for x in res]
                print(f"    {k} ptr {p:#x} saw {t} ref {ref_sum[k]} now {now} (fixed later: {now == ref_sum[k]}) "
                      f"gpu pages/block {gpu_pages}", flush=True)
            seen.clear()
        err = lib.decode_errors(True)
        if err["count"]:
            where = [f"kv layer {j}" for j in range(cfg.n_layers)
                     if m.kv_lease.dptr + j * m.kv_slot == err["stream"]] if m.kv_format != "bf16" else []
            where += [unstaged.get(err["stream"], "?")]
            print(f"  CORRUPT packed chunks: {err['count']} first stream {err['stream']:#x} chunk {err['chunk']} "
                  f"freq sum {err['detail']} {where}", flush=True)

    # Regression guard for the one-time ~47 s stall of round 1 (reuse fences
    # consumed by the first writer, profiles/r2_corrupt_chunk_hunt.md) and for
    # the layout convergence of step 0 (TieredLlama._settle): no early step may
    # take more than --max-ratio x the steady (last) step.
    if len(times) >= 3:
        steady = times[-1]
        worst = max(times[:-1])
        print(f"transient check: worst early step {worst * 1e3:.1f} ms, steady {steady * 1e3:.1f} ms", flush=True)
        if worst > a.max_ratio * steady:
            raise SystemExit(f"transient stall: an early step took {worst / steady:.1f}x the steady step")


if __name__ == "__main__":
    main()
