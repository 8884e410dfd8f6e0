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
        b = torch.load(p, weights_only=True)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        print(f"run {i}: {len(bad)} differ  {info}", flush=True)
        for k in bad:
            print(f"   {k} {tuple(a[k].shape)}: {describe(a[k], b[k])}", flush=True)
        bad_runs += bool(bad)
        os.remove(p)
    print(f"DIAG_DONE bad_runs={bad_runs}/{runs}", flush=True)


if __name__ == "__main__":
    main()
