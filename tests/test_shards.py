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
