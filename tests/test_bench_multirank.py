"""bench.py's multi-GPU path rehearsed on the CPU (fake backend, gloo, 4 ranks
under torch.distributed.run): every rank's runtime manages only its own GPU and
rests its host tier on that GPU's NUMA node; tensor-parallel and peer-shard
(config 4) runs decode the same model as the single-rank run."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--backend", "fake", "--model", "small", "--batch", "8", "--context", "32", "--steps", "1", "--warmup", "1",
        "--weights", "ans", "--kv-format", "bf16", "--oversub", "1.25"]


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(tmp_path, nproc: int, extra: list, force_dist: bool = False) -> tuple[dict, torch.Tensor]:
    dump = str(tmp_path / f"logits_{nproc}_{int(force_dist)}_{'_'.join(extra)}.pt")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", OGKM_UNIT_MIN_MB="0")
    if force_dist:
        env["OGKM_DIST_FORCE"] = "1"
    if nproc == 1 and not force_dist:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
               "--gpus", str(nproc)]
    r = subprocess.run(cmd + ARGS + extra + ["--dump-logits", dump], env=env, capture_output=True, text=True,
                       timeout=900)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(lines[-1]), torch.load(dump)


@pytest.fixture(scope="module")
def single(tmp_path_factory):
    return _bench(tmp_path_factory.mktemp("b1"), 1, [])


@pytest.mark.parametrize("parallel", ["tp", "shards"])
def test_bench_four_ranks(single, tmp_path, parallel):
    one, ref = single
    out, logits = _bench(tmp_path, 4, ["--parallel", parallel])
    cfg = out["config"]
    assert out["n_gpus"] == 4 and cfg["parallelism"] == f"{parallel}4" and cfg["global_batch"] == 8
    # fake_numa_nodes=2: GPUs 0-1 on node 0, 2-3 on node 1 - each rank's host tier follows its GPU
    assert cfg["rank_host_numa_nodes"] == [0, 0, 1, 1]
    assert logits.shape == ref.shape
    if parallel == "shards":
        # the same single-GPU math on each rank's own sequences: bit-identical
        assert torch.equal(logits, ref)
    else:
        # row-parallel partial sums are reduced in a different order
        torch.testing.assert_close(logits, ref, atol=0.05, rtol=0.05)


@pytest.mark.parametrize("parallel", ["tp", "shards"])
def test_bench_forced_one_rank_group(single, tmp_path, parallel):
    """OGKM_DIST_FORCE=1: a one-rank process group in which every collective
    still runs (the GPU twin is tests/test_gpu_rccl.py) - bit-identical."""
    _, ref = single
    out, logits = _bench(tmp_path, 1, ["--parallel", parallel], force_dist=True)
    assert out["n_gpus"] == 1
    assert torch.equal(logits, ref)


@pytest.mark.parametrize("parallel", ["tp", "shards"])
def test_plan_traffic_matches_measured_four_ranks(tmp_path, parallel):
    """The plan's per-step traffic (TieredLlama.traffic(), what bench.py
    --plan-only prints) against what a 4-rank run moved: xGMI bytes received by
    the collectives exactly, PCIe (streamed units) within 10%."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", OGKM_UNIT_MIN_MB="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "4"]
    args = list(ARGS)
    args[args.index("--steps") + 1] = "2"
    args += ["--parallel", parallel]
    r = subprocess.run(cmd + args, env=env, capture_output=True, text=True, timeout=900)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-4000:]
    t = json.loads(lines[-1])["aux"]["traffic_per_step_gb"]
    assert t["xgmi_planned"] > 0
    assert abs(t["xgmi_measured"] - t["xgmi_planned"]) <= 1e-6 + 1e-3 * t["xgmi_planned"], t
    assert t["pcie_planned"] > 0 and abs(t["pcie_measured"] - t["pcie_planned"]) <= 0.1 * t["pcie_planned"], t


def test_plan_only_prints_every_configuration():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--plan-only"], capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    plans = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    got = {(p["plan"], p["parallel"]) for p in plans}
    for m in ("llama3-70b", "llama3-405b"):
        for n in (1, 2, 4, 8):
            assert (m, f"tp{n}") in got
            if n > 1:
                assert (m, f"shards{n}") in got
    for p in plans:
        r0 = p["per_rank"]
        assert len(r0["host_numa_node"]) == p["n_gpus"] and r0["cxl_numa_node"] == r0["host_numa_node"]
        assert p["predicted_ms_per_step"] > 0 and r0["pcie_gb_per_step"] >= 0
        if p["n_gpus"] > 1:
            assert r0["xgmi_gb_per_step"] > 0
