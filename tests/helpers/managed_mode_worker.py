"""Worker for tests/test_managed_mode_gpu.py: a stock torch.nn transformer run
either plainly (torch's own allocator, everything resident) or under
``ogkm.managed()`` with its parameters oversubscribing the HBM arena; saves the
outputs / gradients / updated parameters for a bitwise comparison.

    python managed_mode_worker.py plain|managed OUT.pt [--lazy] [--advise] [--pack]
"""
from __future__ import annotations

import os
import resource
import sys
import time

resource.setrlimit(resource.RLIMIT_CORE, (0, 0))  # a crash must not spend minutes writing a core
# BLAS workspaces are allocated inside a GEMM and never passed to an op, so
# they stay resident (pinned) for the process lifetime - one per (thread,
# stream): keep them small next to the 384 MB arena. Same in both runs, so the
# GEMM algorithm choice (and the bits) match.
os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
os.environ.setdefault("HIPBLASLT_WORKSPACE_SIZE", "32768")

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

D, FF, LAYERS, HEADS = 1024, 4096, 16, 16
BATCH, SEQ = 4, 128
ARENA_MB = int(os.environ.get("OGKM_TEST_ARENA_MB", "384"))  # (diagnostics may shrink it)


def build():
    torch.manual_seed(0)
    layer = torch.nn.TransformerEncoderLayer(D, HEADS, FF, dropout=0.0, batch_first=True)
    model = torch.nn.TransformerEncoder(layer, LAYERS, enable_nested_tensor=False)
    x = torch.randn(BATCH, SEQ, D)
    return model, x


def run(model, x, log=False):
    """Inference pass + one training step (forward, backward, SGD)."""
    def say(m):
        if log:
            print(m, flush=True)
    model.eval()
    with torch.no_grad():
        y_inf = model(x)
    say("inference done")
    model.train()
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    y = model(x)
    say("train forward done")
    loss = y.float().pow(2).mean()
    loss.backward()
    say("backward done")
    if os.environ.get("OGKM_DIAG_SNAP_OUT"):  # (diagnostics) a gradient's value right after backward
        w = dict(model.named_parameters())[os.environ["OGKM_DIAG_SNAP"]]
        torch.save(w.grad.detach().cpu().clone(), os.environ["OGKM_DIAG_SNAP_OUT"])
    opt.step()
    say("step done")
    if os.environ.get("OGKM_DIAG_SNAP2_OUT"):  # (diagnostics) the same gradient right after the step
        w = dict(model.named_parameters())[os.environ["OGKM_DIAG_SNAP"]]
        torch.save(w.grad.detach().cpu().clone(), os.environ["OGKM_DIAG_SNAP2_OUT"])
    if os.environ.get("OGKM_DIAG_RES"):  # (diagnostics) chunks owned by two tensors' blocks
        _chunk_owners(model, "after step")
    out = {"y_inf": y_inf, "loss": loss.detach()}
    for name, p in model.named_parameters():
        out["p." + name] = p.detach()
        out["g." + name] = p.grad.detach()
    if os.environ.get("OGKM_DIAG_STABLE") and "ogkm" in sys.modules:  # (diagnostics, managed run only)
        from ogkm._native import lib

        res = {}
        for k, v in out.items():
            res[k] = v.cpu()
            if os.environ.get("OGKM_DIAG_SECOND_OUT") and k == "g." + os.environ.get("OGKM_DIAG_SNAP", ""):
                torch.cuda.synchronize()
                torch.save(v.cpu().clone(), os.environ["OGKM_DIAG_SECOND_OUT"])  # the same tensor copied out again
            if os.environ.get("OGKM_DIAG_OWN"):
                bad = lib.check_ownership()
                if bad:
                    print(f"OWNERSHIP after {k}: {bad[:600]}", flush=True)
            rid = lib.torch_managed_range_id(v.untyped_storage().data_ptr(), 0)
            if not rid:
                continue
            for b in range((v.untyped_storage().nbytes() + (2 << 20) - 1) >> 21):
                ri = lib.residency_info(rid, b << 21)
                gpu = [e for e in ri["resident_on"] if e.get("tier") == "hbm" or e.get("kind") == "gpu" or "gpu" in str(e)]
                if gpu and ri["stable_chunk"] >= 0 and all(e["chunk"] != ri["stable_chunk"] for e in gpu):
                    print(f"STABLE_MISMATCH {k}[{b}] stable_chunk {ri['stable_chunk']} resident {gpu}", flush=True)
        return res
    if os.environ.get("OGKM_DIAG_PINNED_CPU"):  # (diagnostics) copy-outs into pinned host memory
        return {k: torch.empty(v.shape, dtype=v.dtype, pin_memory=True).copy_(v) for k, v in out.items()}
    return {k: v.cpu() for k, v in out.items()}


def _chunk_owners(model, when):
    from ogkm._native import lib

    owners = {}
    for name, p in model.named_parameters():
        for kind, t in (("p", p), ("g", p.grad)):
            if t is None:
                continue
            rid = lib.torch_managed_range_id(t.untyped_storage().data_ptr(), 0)
            if not rid:
                continue
            for b in range((t.untyped_storage().nbytes() + (2 << 20) - 1) >> 21):
                ri = lib.residency_info(rid, b << 21)
                for e in ri["resident_on"]:
                    key = (str(sorted((k, v) for k, v in e.items() if k not in ("pages", "encoded_bytes"))))
                    owners.setdefault(key, []).append(f"{kind}.{name}[{b}]")
    dup = {k: v for k, v in owners.items() if len(v) > 1}
    print(f"CHUNK_OWNERS {when}: {len(owners)} chunks, {len(dup)} shared", flush=True)
    for k, v in list(dup.items())[:10]:
        print(f"   {k}: {v}", flush=True)


def main() -> None:
    which, path = sys.argv[1], sys.argv[2]
    if which == "plain":
        model, x = build()
        res = run(model.cuda(), x.cuda())
        torch.cuda.synchronize()
        torch.save(res, path)
        print("PLAIN_OK", len(res))
        return
    import faulthandler
    import threading

    import ogkm
    from ogkm import allocator, rt

    # Hang diagnostics (stderr): Python stacks after 60 s, ring progress every 10 s.
    faulthandler.dump_traceback_later(60, exit=False)

    def watchdog():
        while True:
            time.sleep(10)
            try:
                rings = [(r["kind"], r["submitted"], r["completed"]) for r in rt.stats()["rings"] if r["dev"] == 0]
                print("WATCHDOG", round(time.perf_counter() - t0, 1), rings, file=sys.stderr, flush=True)
            except Exception as e:  # noqa: BLE001
                print("WATCHDOG error", e, file=sys.stderr, flush=True)

    t0 = time.perf_counter()
    threading.Thread(target=watchdog, daemon=True).start()

    allocator.enable(managed_min_mb=1)
    rt.init("hip", hbm_budget={0: ARENA_MB << 20}, stable_lazy_unmap=int("--lazy" in sys.argv))
    model, x = build()
    param_bytes = sum(p.numel() * p.element_size() for p in model.parameters())
    mode = ogkm.managed()
    t0 = time.perf_counter()
    advised = 0
    with mode:
        model = model.cuda()
        print("model on gpu", flush=True)
        if "--advise" in sys.argv:
            # Every 4th weight prefers host DRAM and is accessed_by the GPU: the
            # runtime decides to access it remotely once it rests in host DRAM,
            # which the stable VA cannot map - served by a local copy instead.
            from ogkm._native import lib

            for i, p in enumerate(model.parameters()):
                if i % 4 == 0 and allocator.is_managed(p):
                    allocator.set_read_mostly(p, on=False)
                    allocator.advise(p, rt.ADVISE_SET_PREFERRED_LOCATION, f"host:{lib.host_node()}")
                    allocator.advise(p, rt.ADVISE_SET_ACCESSED_BY, proc=0)
                    advised += 1
        if "--pack" in sys.argv:
            # one inference pass first: the weights' GPU copies are dropped
            # clean, the runtime packs their host copies (ANS1); the measured
            # pass below refills them from the packed bytes (DECODE_ANS)
            from ogkm._native import lib

            model.eval()
            for _ in range(2):
                with torch.no_grad():
                    model(x.cuda())
                torch.cuda.synchronize()
                lib.pack_wait(60000)
        res = run(model, x.cuda(), log=True)
        if os.environ.get("OGKM_DIAG_RES"):
            _chunk_owners(model, "after copy-out")
        if os.environ.get("OGKM_DIAG_HOSTREAD_OUT"):  # (diagnostics) the runtime's host-side view of a gradient
            from ogkm._native import lib

            g = dict(model.named_parameters())[os.environ["OGKM_DIAG_SNAP"]].grad
            st = g.untyped_storage()
            rid = lib.torch_managed_range_id(st.data_ptr(), 0)
            buf = torch.empty(st.nbytes(), dtype=torch.uint8)
            lib.read(rid, 0, buf.data_ptr(), st.nbytes(), -1)
            torch.save(buf.view(g.dtype).view(g.shape).clone(), os.environ["OGKM_DIAG_HOSTREAD_OUT"])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    from ogkm._native import lib

    own = lib.check_ownership()  # every residency's chunk owned by its block, none shared
    assert own == "", own[:2000]
    torch.save(res, path)
    st = rt.stats()
    print("MANAGED_OK", {"param_mb": param_bytes >> 20, "arena_mb": ARENA_MB, "ops": mode.ops,
                         "faulted_ops": mode.faulted_ops, "prefetches": mode.prefetches,
                         "evictions": st["evictions"], "htd_mb": st["bytes_xfer_htd"] >> 20,
                         "dth_mb": st["bytes_xfer_dth"] >> 20, "vmm_remaps": st["vmm_remaps"],
                         "tlb_flushes": st["tlb_flushes"], "vmm_errors": st["vmm_errors"], "seconds": round(dt, 3),
                         "advised": advised, "remote_fallbacks": st["remote_fallbacks"],
                         "write_invalidations": st["write_invalidations"], "packed_blocks": st["packed_blocks"],
                         "packed_decodes": st["packed_decodes"], "pack_expansions": st["pack_expansions"]})


if __name__ == "__main__":
    main()
