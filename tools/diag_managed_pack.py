"""Repeat the packed-host-copy transparent-mode run (tests/test_managed_mode_gpu.py
::test_packed_host_copies_run_bitwise_under_managed_mode) and describe every
difference from the plain run: which tensors, how many elements, and which
4 KB pages / 2 MB blocks of the tensor they fall in (a copy or decode fault
shows up as whole pages or 64 KB segments; a numeric difference is spread out).

    python tools/diag_managed_pack.py OUT_DIR RUNS [extra worker args...]
"""
from __future__ import annotations

import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(os.path.dirname(HERE), "tests", "helpers", "managed_mode_worker.py")


def run(args):
    r = subprocess.run([sys.executable, WORKER] + args, capture_output=True, text=True, timeout=150,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-3000:], flush=True)
        raise SystemExit(f"worker rc={r.returncode}")
    return r.stdout


def describe(a: torch.Tensor, b: torch.Tensor) -> str:
    fa, fb = a.reshape(-1), b.reshape(-1)
    ne = (fa != fb).nonzero().reshape(-1)
    esz = a.element_size()
    pages = sorted({int(i) * esz >> 12 for i in ne})
    blocks = sorted({p >> 9 for p in pages})
    d = (fa.double() - fb.double()).abs()
    rel = (d / fa.double().abs().clamp_min(1e-30))[ne]
    return (f"{ne.numel()}/{fa.numel()} elems differ, pages {len(pages)} (first {pages[:6]}, last {pages[-3:]}), "
            f"blocks {blocks[:8]}, max abs {d.max().item():.3e}, median rel {rel.median().item():.3e}, "
            f"zeros in managed {(fb[ne] == 0).sum().item()}")


def page_sources(a, b, k):
    """Where the wrong 4 KB pages of b[k] come from: the same page (or any page)
    of the initial / updated weights and gradients of the plain run."""
    sys.path.insert(0, os.path.dirname(WORKER))
    import managed_mode_worker as w
    model, _ = w.build()
    init = {"init." + n: p.detach() for n, p in model.named_parameters()}
    cands = dict(init)
    cands.update({n: t for n, t in a.items() if n.startswith(("p.", "g."))})
    esz = a[k].element_size()
    per = 4096 // esz
    fa, fb = a[k].reshape(-1), b[k].reshape(-1)
    bad = [p for p in range(fa.numel() // per) if not torch.equal(fa[p * per:(p + 1) * per], fb[p * per:(p + 1) * per])]
    index = {}
    for n, t in cands.items():
        if t.element_size() != esz:
            continue
        ft = t.reshape(-1)
        for q in range(ft.numel() // per):
            index.setdefault(ft[q * per:(q + 1) * per].numpy().tobytes(), (n, q))
    hits = {}
    for p in bad:
        src = index.get(fb[p * per:(p + 1) * per].numpy().tobytes())
        key = "none" if src is None else f"{src[0]} ({'same page' if src[1] == p else f'page {src[1]} vs {p}'})"
        key = key if src is None or src[1] == p else f"{src[0]} (other page, offset {src[1] - p:+d})"
        hits[key] = hits.get(key, 0) + 1
    return dict(sorted(hits.items(), key=lambda x: -x[1])[:6])


def main():
    out, runs, extra = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    os.makedirs(out, exist_ok=True)
    ref = os.path.join(out, "plain.pt")
    print(run(["plain", ref]).strip().splitlines()[-1], flush=True)
    a = torch.load(ref, weights_only=True)
    bad_runs = 0
    for i in range(runs):
        p = os.path.join(out, f"managed{i}.pt")
        log = run(["managed", p, "--pack"] + extra)
        info = log.split("MANAGED_OK", 1)[1].strip().splitlines()[0]
        for line in log.splitlines():
            if line.startswith(("CHUNK_OWNERS", "   (", "STABLE_MISMATCH", "OWNERSHIP")) or line.startswith("   [("):
                print(line[:300], flush=True)
        b = torch.load(p, weights_only=True)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        print(f"run {i}: {len(bad)} differ  {info}", flush=True)
        snap = os.environ.get("OGKM_DIAG_SNAP_OUT")
        if snap and os.path.exists(snap):
            k = "g." + os.environ["OGKM_DIAG_SNAP"]
            s = torch.load(snap, weights_only=True)
            print(f"   after backward {k}: " + ("equal" if torch.equal(a[k], s) else describe(a[k], s)), flush=True)
            os.remove(snap)
        sc = os.environ.get("OGKM_DIAG_SECOND_OUT")
        if sc and os.path.exists(sc):
            k = "g." + os.environ["OGKM_DIAG_SNAP"]
            s = torch.load(sc, weights_only=True)
            print(f"   second copy-out of {k}: " + ("equal" if torch.equal(a[k], s) else describe(a[k], s))
                  + ("; first copy-out equal" if torch.equal(a[k], b[k]) else "; first copy-out differs"), flush=True)
            os.remove(sc)
        hr = os.environ.get("OGKM_DIAG_HOSTREAD_OUT")
        if hr and os.path.exists(hr):
            k = "g." + os.environ["OGKM_DIAG_SNAP"]
            s = torch.load(hr, weights_only=True)
            print(f"   runtime read of {k} at the end: " + ("equal" if torch.equal(a[k], s) else describe(a[k], s)), flush=True)
            os.remove(hr)
        snap2 = os.environ.get("OGKM_DIAG_SNAP2_OUT")
        if snap2 and os.path.exists(snap2):
            k = "g." + os.environ["OGKM_DIAG_SNAP"]
            s = torch.load(snap2, weights_only=True)
            print(f"   after step {k}: " + ("equal" if torch.equal(a[k], s) else describe(a[k], s)), flush=True)
            os.remove(snap2)
        for k in bad:
            print(f"   {k} {tuple(a[k].shape)}: {describe(a[k], b[k])}", flush=True)
            print(f"      wrong pages match: {page_sources(a, b, k)}", flush=True)
        bad_runs += bool(bad)
        os.remove(p)
    print(f"DIAG_DONE bad_runs={bad_runs}/{runs}", flush=True)


if __name__ == "__main__":
    main()
