"""GPU peer topology: link types, peer access, NUMA / CXL locality, and the
sizing rules that follow from them.

Reference: peer capabilities come from RM (`p2pGetCaps`
src/nvidia/src/kernel/platform/p2p/p2p_caps.c:69-121; UVM `parent_peers_init`
kernel-open/nvidia-uvm/uvm_gpu.c:2332-2388) with link types PCIe/NVLink1-5/C2C
(uvm_gpu.h:613-620), and the CXL fork adds a CXL connectivity bit that nothing
produces (ctrl0000system.h:1085-1147, p2p_caps.h:35).

MI355X: the link type comes from ``hipExtGetLinkTypeAndHopCount`` (xGMI vs
PCIe), access from ``hipDeviceCanAccessPeer``; CXL reachability per GPU is the
CXL pool's NUMA distance from the GPU's NUMA node (cxl.p2p_caps). An 8-GPU
MI355X node is fully connected: 7 point-to-point xGMI links per GPU, so
  * a ring collective is bound by ONE link per hop (~153 GB/s per direction),
  * a direct all-gather / all-to-all uses all 7 links at once (~1 TB/s in),
  * every message pays a fixed latency, so buckets must be large enough that
    the latency term stays a small fraction of the wire time.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

from .._native import lib

LINK_NONE, LINK_SELF, LINK_PCIE, LINK_XGMI = 0, 1, 2, 3
LINK_NAMES = {LINK_NONE: "none", LINK_SELF: "self", LINK_PCIE: "pcie", LINK_XGMI: "xgmi"}

# Per-direction planning numbers (MI355X node; measured values override them).
XGMI_LINK_GBPS = 153.0
PCIE_GBPS = 57.0          # measured H2D on the box (profiles/probe_host_r1.txt)
COLLECTIVE_LATENCY_US = 12.0


@dataclass
class PeerTopology:
    n: int
    link: list = field(default_factory=list)      # link[a][b] in LINK_*
    access: list = field(default_factory=list)    # access[a][b] = a can map b's memory
    numa: list = field(default_factory=list)      # GPU -> host NUMA node
    cxl: dict = field(default_factory=dict)       # GPU -> cxl.p2p_caps() dict
    measured_gbps: dict = field(default_factory=dict)  # (a, b) -> GB/s when measured

    # ---------------------------------------------------------------- discovery
    @staticmethod
    def discover() -> "PeerTopology":
        n = lib.device_count()
        t = PeerTopology(n)
        t.link = [[lib.link_type(a, b) for b in range(n)] for a in range(n)]
        t.access = [[a != b and bool(lib.can_access_peer(a, b)) for b in range(n)] for a in range(n)]
        t.numa = [lib.device_numa_node(a) for a in range(n)]
        try:
            from .. import cxl

            t.cxl = {a: cxl.p2p_caps(a) for a in range(n)}
        except Exception:  # no CXL registry (e.g. runtime without CXL discovery)
            t.cxl = {}
        return t

    def enable_all_peers(self) -> int:
        """Enable peer access on every pair that supports it (uvm_va_space.c:1169
        enable_peers analog). Returns the number of enabled directed pairs."""
        k = 0
        for a in range(self.n):
            for b in range(self.n):
                if self.access[a][b]:
                    lib.enable_peer(a, b)
                    k += 1
        return k

    # ---------------------------------------------------------------- queries
    def link_name(self, a: int, b: int) -> str:
        return LINK_NAMES.get(self.link[a][b], "?")

    def fully_connected_xgmi(self) -> bool:
        return all(self.link[a][b] == LINK_XGMI for a in range(self.n) for b in range(self.n) if a != b)

    def peer_gbps(self, a: int, b: int) -> float:
        if (a, b) in self.measured_gbps:
            return self.measured_gbps[(a, b)]
        lt = self.link[a][b]
        return {LINK_XGMI: XGMI_LINK_GBPS, LINK_PCIE: PCIE_GBPS, LINK_SELF: float("inf")}.get(lt, 0.0)

    def p2p_caps(self, a: int, b: int) -> dict:
        """Per-pair capability record (NV0000_CTRL_SYSTEM_GET_P2P_CAPS analog)."""
        caps = {
            "link": self.link_name(a, b),
            "read": self.access[a][b],
            "write": self.access[a][b],
            "atomics": self.link[a][b] == LINK_XGMI,
            "gbps": self.peer_gbps(a, b),
        }
        if a in self.cxl:
            caps["cxl_reachable"] = bool(self.cxl[a].get("cxl_supported", False))
        return caps

    def ring_order(self, ranks: Optional[list] = None) -> list:
        """A ring over ``ranks`` that only uses xGMI hops when possible
        (greedy nearest neighbour; identity on a fully connected node)."""
        ranks = list(range(self.n)) if ranks is None else list(ranks)
        if not ranks:
            return []
        order, left = [ranks[0]], set(ranks[1:])
        while left:
            cur = order[-1]
            nxt = min(left, key=lambda r: (self.link[cur][r] != LINK_XGMI, r))
            order.append(nxt)
            left.remove(nxt)
        return order

    # ---------------------------------------------------------------- sizing rules
    def allgather_seconds(self, nbytes: int, world: int, algo: str = "direct") -> float:
        """Wire-time model of an all-gather of ``nbytes`` total over ``world`` GPUs.
        ring: world-1 steps, each moving nbytes/world over one link.
        direct: every GPU pulls its world-1 shards over world-1 links at once."""
        if world <= 1:
            return 0.0
        shard = nbytes / world
        bw = XGMI_LINK_GBPS * 1e9
        lat = COLLECTIVE_LATENCY_US * 1e-6
        if algo == "ring":
            return (world - 1) * (shard / bw + lat)
        return shard / bw + lat

    def bucket_bytes(self, world: int, latency_fraction: float = 0.05) -> int:
        """Smallest ring-collective bucket whose per-hop latency stays below
        ``latency_fraction`` of its wire time, rounded to 2 MB."""
        if world <= 1:
            return 0
        bw = XGMI_LINK_GBPS * 1e9
        lat = COLLECTIVE_LATENCY_US * 1e-6
        per_hop = lat / latency_fraction * bw  # bytes each hop must carry
        total = per_hop * world
        return int(-(-total // (2 << 20)) * (2 << 20))

    def choose_tp(self, weight_bytes: int, hbm_bytes_per_gpu: int, candidates=(1, 2, 4, 8),
                  reserve_fraction: float = 0.15) -> int:
        """Smallest TP degree whose weight shard fits HBM (minus a reserve for
        KV / activations); the largest candidate when none fits (then the
        tiering runtime oversubscribes)."""
        usable = hbm_bytes_per_gpu * (1.0 - reserve_fraction)
        for tp in candidates:
            if tp <= max(self.n, 1) and weight_bytes / tp <= usable:
                return tp
        return max(c for c in candidates if c <= max(self.n, 1))

    def to_dict(self) -> dict:
        return {
            "n": self.n,
            "links": [[self.link_name(a, b) for b in range(self.n)] for a in range(self.n)],
            "access": self.access,
            "numa": self.numa,
            "fully_connected_xgmi": self.fully_connected_xgmi() if self.n > 1 else None,
            "cxl": {str(k): v for k, v in self.cxl.items()},
        }


def discover() -> PeerTopology:
    return PeerTopology.discover()
