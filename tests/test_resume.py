"""In-place resume of a decoding model (FBSR restores VRAM in
place, fbsr.c:37-104; suspend/resume keeps VA spaces, uvm_global.c:272-415):
process A checkpoints a TieredLlama mid-decode (residency map with data +
sidecar), process B restores every managed range under its recorded id and
VAs and the next decode step's logits are bit-identical to A's."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "helpers", "resume_worker.py")


def _run(args):
    r = subprocess.run([sys.executable, WORKER] + args, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _resume(tmp_path, backend, wf, kf):
    _run(["save", str(tmp_path), backend, wf, kf])
    out = _run(["restore", str(tmp_path), backend, wf, kf])
    res = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert res["identical"], res
    assert res["ranges"] > 10


@pytest.mark.parametrize("wf,kf", [("bf16", "bf16"), ("ans", "ans")])
def test_resume_in_place_fake(tmp_path, wf, kf):
    _resume(tmp_path, "fake", wf, kf)


@pytest.mark.gpu
@pytest.mark.parametrize("wf,kf", [("bf16", "bf16"), ("ans", "ans")])
def test_resume_in_place_gpu(tmp_path, wf, kf):
    _resume(tmp_path, "hip", wf, kf)
