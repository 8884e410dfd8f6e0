"""Parallelism: RCCL process groups (comm), tensor parallel (tp), peer-shard
weights over xGMI (shards), and GPU peer topology (topology)."""
from . import comm, tp, topology, shards  # noqa: F401
