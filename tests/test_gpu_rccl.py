"""RCCL on one GPU: bench.py under torch.distributed.run with a one-rank "nccl"
process group (OGKM_DIST_FORCE=1), so every collective of the multi-GPU decode
path really runs through RCCL - tensor-parallel all-reduces / vocab all-gather
and the peer-shard all-gathers, on the compute and side streams beside the
runtime's rings. Logits must equal the plain single-process run. (8-GPU runs
are the driver's; this is the part of that path one GPU can execute.)"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "small", "--batch", "8", "--context", "64", "--steps", "2", "--warmup", "1", "--no-aux",
        "--weights", "ans", "--kv-format", "bf16",
        "--oversub", "1.5"]


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, dist: bool, extra: list) -> tuple[dict, torch.Tensor]:
    dump = str(tmp_path / f"logits_{int(dist)}_{'_'.join(extra)}.pt")
    env = dict(os.environ, PYTHONPATH=ROOT, OGKM_UNIT_MIN_MB="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")]
    if dist:
        env["OGKM_DIST_FORCE"] = "1"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "1"]
    r = subprocess.run(cmd + ARGS + extra + ["--dump-logits", dump], env=env, capture_output=True, text=True,
                       timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(lines[-1]), torch.load(dump)


@pytest.mark.parametrize("parallel", ["tp", "shards"])
def test_rccl_one_rank_matches_single_process(tmp_path, parallel):
    _, ref = _run(tmp_path, False, ["--parallel", parallel])
    out, logits = _run(tmp_path, True, ["--parallel", parallel])
    assert out["n_gpus"] == 1
    assert torch.equal(logits, ref)
