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
import time

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


def _bench(tmp_path, nproc: int, extra: list, force_dist: bool = False,
           self_launch: bool = False, env_extra: dict | None = None) -> tuple[dict, torch.Tensor]:
    tag = "_env" if env_extra else ""
    dump = str(tmp_path / f"logits_{nproc}_{int(force_dist)}_{int(self_launch)}_{'_'.join(extra)}{tag}.pt")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", OGKM_UNIT_MIN_MB="0", **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    if force_dist:
        env["OGKM_DIST_FORCE"] = "1"
    if self_launch:  # bench.py spawns its own rank processes (no torchrun)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc)]
    elif nproc == 1 and not force_dist:
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


@pytest.fixture(scope="module")
def torchrun_tp4(tmp_path_factory):
    return _bench(tmp_path_factory.mktemp("tr4"), 4, ["--parallel", "tp"])


@pytest.mark.parametrize("parallel", ["tp", "shards"])
def test_bench_four_ranks(single, torchrun_tp4, tmp_path, parallel):
    one, ref = single
    out, logits = torchrun_tp4 if parallel == "tp" else _bench(tmp_path, 4, ["--parallel", parallel])
    cfg = out["config"]
    assert out["n_gpus"] == 4 and cfg["parallelism"] == f"{parallel}4" and cfg["global_batch"] == 8
    assert cfg["rccl_world"] == 4 and cfg["launcher"] == "external"
    # fake_numa_nodes=2: GPUs 0-1 on node 0, 2-3 on node 1 - each rank's host tier follows its GPU
    assert cfg["rank_host_numa_nodes"] == [0, 0, 1, 1]
    assert logits.shape == ref.shape
    if parallel == "shards":
        # the same single-GPU math on each rank's own sequences: bit-identical
        assert torch.equal(logits, ref)
    else:
        # row-parallel partial sums are reduced in a different order (bf16
        # activations between the GEMMs): measured max |diff| 0.023, mean 0.0044
        # on logits of magnitude ~3; the greedy tokens agree wherever the
        # 1-rank top-2 margin exceeds twice the worst difference
        torch.testing.assert_close(logits, ref, atol=0.03, rtol=0.01)
        assert (logits.float() - ref.float()).abs().mean() < 0.01
        top2 = ref.float().topk(2, dim=-1).values
        clear = (top2[:, 0] - top2[:, 1]) > 0.05
        assert torch.equal(logits.argmax(-1)[clear], ref.argmax(-1)[clear])


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
    the collectives exactly, PCIe (streamed units) within 10% - under the static
    plan, whose residency the traffic model describes (planner off, the
    bench default, decides residency at run time: tests/test_model.py)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", OGKM_UNIT_MIN_MB="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "4"]
    args = list(ARGS)
    args[args.index("--steps") + 1] = "2"
    args += ["--parallel", parallel, "--planner", "static"]
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


def test_bench_self_launch_four_ranks(single, torchrun_tp4, tmp_path):
    """``bench.py --gpus 4`` without torchrun spawns 4 rank processes itself:
    a real 4-rank job whose logits equal the torchrun run's bit for bit."""
    out, logits = _bench(tmp_path, 4, ["--parallel", "tp"], self_launch=True)
    cfg = out["config"]
    assert out["n_gpus"] == 4 and cfg["rccl_world"] == 4 and cfg["launcher"] == "bench.py"
    assert cfg["parallelism"] == "tp4" and cfg["rank_host_numa_nodes"] == [0, 0, 1, 1]
    assert torch.equal(logits, torchrun_tp4[1])
    one, _ = single
    assert one["n_gpus"] == 1 and one["config"]["rccl_world"] == 1 and one["config"]["launcher"] == "none"


def _launch(extra_env: dict, extra_args: list, timeout: float):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", OGKM_UNIT_MIN_MB="0", **extra_env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"] + ARGS + extra_args
    t0 = time.monotonic()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    return r, time.monotonic() - t0


def test_bench_launcher_child_failure_stops_job():
    """One rank dies after joining the group: the launcher kills the other
    three (blocked in a collective) and exits non-zero, without a JSON line."""
    r, dt = _launch({"OGKM_BENCH_FAIL_RANK": "1"}, ["--launch-timeout", "600"], timeout=300)
    assert r.returncode != 0 and "rank 1 exited with status 3" in r.stderr, r.stderr[-3000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert dt < 200


@pytest.mark.parametrize("where", ["init", "step"])
def test_bench_launcher_timeout_kills_hung_rank(where):
    """A rank that stops making progress: on the launch timeout the launcher
    SIGUSR1s every rank - each prints all its threads' Python stacks and the
    runtime's rings / leases (ogkm.diag) - then kills the job (exit 124)."""
    timeout = "20" if where == "init" else "60"
    args = ["--launch-timeout", timeout] + (["--warmup", "2"] if where == "step" else [])
    r, dt = _launch({"OGKM_BENCH_HANG_RANK": "2", "OGKM_BENCH_HANG_AT": where, "OGKM_HANG_DUMP_WAIT_S": "5"},
                    args, timeout=300)
    err = r.stderr
    assert r.returncode == 124 and "killing all 4" in err, err[-3000:]
    assert dt < 180
    # every rank dumped; the hung one shows where it sleeps
    for rank in range(4):
        assert f"[ogkm-hang] rank {rank} pid" in err, err[-5000:]
    assert err.count("[ogkm-hang]") >= 8  # a header and an end line per rank
    assert "time.sleep" in err or "in main" in err, err[-5000:]
    assert "[ogkm-dump]" in err
    if where == "step":
        # the runtime is up on the hung rank: its rings and leases are listed
        assert "ring cpu_to_gpu/" in err and "leases outstanding" in err, err[-5000:]


@pytest.mark.parametrize("ws,gpus", [("2", "4"), ("4", "1"), ("1", "2")])
def test_bench_refuses_world_size_mismatch(ws, gpus):
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE=ws, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", gpus] + ARGS, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr, r.stderr[-2000:]


def test_shards_two_ranks_planner_off_small_arena(single, tmp_path):
    """Peer shards under the default runtime-decided residency (planner off,
    next-use hints) on a small fake HBM (forced evictions while gathers are in
    flight): the 2-rank job completes - the configuration that hung on the GPU
    in round 4 - and decodes the single-rank logits bit for bit."""
    _, ref = single
    out, logits = _bench(tmp_path, 2, ["--parallel", "shards", "--planner", "off", "--oversub", "2.0", "--fake-hbm-mb", "96",
                                       "--launch-timeout", "300"], self_launch=True)
    cfg = out["config"]
    assert cfg["planner"] == "off" and cfg["parallelism"] == "shards2"
    assert out["aux"]["evictions"] > 0
    assert torch.equal(logits, ref)


def test_shards_two_ranks_read_duplicates(tmp_path):
    """Peer shards with HBM to spare (oversub 0.4: 2.5x the rank's shard
    footprint): every gathered unit stays on each rank as a read duplicate
    after its first gather; the decode is bit-exact against the same job
    re-gathering every unit (OGKM_GATHER_CACHE_MB=0)."""
    args = ["--parallel", "shards", "--oversub", "0.4", "--launch-timeout", "300", "--steps", "3"]
    out, logits = _bench(tmp_path, 2, args, self_launch=True)
    base, ref = _bench(tmp_path, 2, args, self_launch=True, env_extra={"OGKM_GATHER_CACHE_MB": "0"})
    assert out["config"]["gather_cache_gb_per_gpu"] > 0 and base["config"]["gather_cache_gb_per_gpu"] == 0
    assert torch.equal(logits, ref)


@pytest.fixture(scope="module")
def single_kv8(tmp_path_factory):
    return _bench(tmp_path_factory.mktemp("k1"), 1, ["--model", "small-kv8"])


@pytest.mark.parametrize("parallel", ["tp", "shards"])
def test_bench_eight_ranks_one_kv_head_per_rank(single_kv8, tmp_path, parallel):
    """The driver's N=8 job rehearsed on the CPU: 8 rank processes under
    torch.distributed.run (fake backend, gloo), a model with 8 KV heads so tp8
    runs ONE KV head per rank (the per-rank shape of 70B / 405B tp8), 8
    packer / ring / fault-thread sets and one node ledger shared by 8
    processes - which a crashed earlier job left behind (a dead pid holding a
    slot and 300 MB). Logits match the 1-rank run: bit-identical for shards
    (each rank decodes its own sequences), within the row-parallel reduction
    order for tp."""
    _, ref = single_kv8
    ledger = str(tmp_path / "ledger")
    worker = os.path.join(ROOT, "tests", "helpers", "ledger_attach_worker.py")
    subprocess.run([sys.executable, worker, "--die", str(300 << 20)], check=True, timeout=120,
                   env=dict(os.environ, OGKM_NODE_LEDGER=ledger, PYTHONPATH=ROOT))
    out, logits = _bench(tmp_path, 8, ["--parallel", parallel, "--model", "small-kv8"],
                         env_extra={"OGKM_NODE_LEDGER": ledger})
    cfg = out["config"]
    assert out["n_gpus"] == 8 and cfg["parallelism"] == f"{parallel}8" and cfg["rccl_world"] == 8
    assert cfg["rank_host_numa_nodes"] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert logits.shape == ref.shape
    if parallel == "shards":
        assert torch.equal(logits, ref)
    else:
        # 8-way row-parallel sums in another order over 16 layers of bf16
        # activations: measured max |diff| 0.034 (1 of 32768 logits past 0.03)
        torch.testing.assert_close(logits, ref, atol=0.06, rtol=0.01)
        assert (logits.float() - ref.float()).abs().mean() < 0.01
        top2 = ref.float().topk(2, dim=-1).values
        clear = (top2[:, 0] - top2[:, 1]) > 0.1
        assert torch.equal(logits.argmax(-1)[clear], ref.argmax(-1)[clear])
    # every rank detached: the stale job's reservation is gone, nothing leaked
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from ogkm._native import lib\n"
            "assert lib.ledger_attach()\n"
            "v = lib.node_ledger(2)['nodes']\n"
            "assert v[0]['reserved'] == 0 and v[1]['reserved'] == 0, v\n"
            "lib.ledger_detach()\n") % ROOT
    subprocess.run([sys.executable, "-c", code], check=True, timeout=120, env=dict(os.environ, OGKM_NODE_LEDGER=ledger))
