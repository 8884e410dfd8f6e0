"""Peer-shard weights: each rank owns 1/W of every layer,
layers are all-gathered with look-ahead before use. CPU: gloo, world 2."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import torch

from ogkm import rt
from ogkm.parallel import shards, topology

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_single_rank_pipeline(fake_rt):
    specs = [shards.LayerSpec(["w"], [(100, 3)]), shards.LayerSpec(["x", "y"], [(5,), (6, 7)])]
    sw = shards.ShardedWeights(specs, torch.bfloat16, rank=0, world=1)
    ref = [{"w": torch.randn(100, 3).bfloat16()}, {"x": torch.randn(5).bfloat16(), "y": torch.randn(6, 7).bfloat16()}]
    for i in range(2):
        sw.load_named(i, ref[i])
    p = shards.ShardGatherPipeline(sw, depth=2)
    for _ in range(3):
        assert torch.equal(p.get(0)["w"], ref[0]["w"])
        l1 = p.get(1)
        assert torch.equal(l1["x"], ref[1]["x"]) and torch.equal(l1["y"], ref[1]["y"])
    p.drain()
    sw.free()


def test_two_rank_gather_gloo():
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests/helpers/shard_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    res = [json.loads(l.split(" ", 1)[1]) for l in r.stdout.splitlines() if l.startswith("SHARDRESULT ")]
    assert len(res) == 2, r.stdout[-2000:] + r.stderr[-4000:]
    assert all(x["ok"] for x in res)
    assert all(x["gathers"] == 6 for x in res)
    # each rank stores about half of the padded weights
    total = (33 * 17 + 17 * 9 + 65 * 31 + 7 + 128 * 3 + 25) * 2
    assert all(abs(x["shard_bytes"] - total / 2) < 16 for x in res)


def test_topology_fake(fake_rt):
    t = topology.discover()
    assert t.n == 2 and t.link_name(0, 1) == "xgmi" and t.link_name(0, 0) == "self"
    assert t.fully_connected_xgmi()
    assert t.enable_all_peers() == 2
    caps = t.p2p_caps(0, 1)
    assert caps["read"] and caps["atomics"] and caps["gbps"] > 100
    assert t.ring_order() == [0, 1]
    # sizing rules: direct all-gather beats ring on a fully connected node
    assert t.allgather_seconds(1 << 30, 8, "direct") < t.allgather_seconds(1 << 30, 8, "ring")
    b = t.bucket_bytes(8)
    assert b % (2 << 20) == 0 and b >= 16 << 20
    # 70B bf16 (141 GB) on 288 GB parts fits at TP=1; 405B (810 GB) needs TP=4
    assert t.choose_tp(141 << 30, 288 << 30) == 1 or t.n < 2
    d = t.to_dict()
    assert d["links"][0][1] == "xgmi"
