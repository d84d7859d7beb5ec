"""Synthetic kwok workloads (SURVEY.md §8(d) / BASELINE.json configs), built
vectorised with numpy so 1M-node / 10M-pod fleets ingest in seconds.

Shapes follow the reference's own benchmark objects
(test/kwokctl/kwokctl_benchmark_test.sh:71-117): nodes `node-%07d`
(ManageAllNodes, empty status), pods with one container
{name: fake-pod, image: fake}, 10 pods per node, ingested Pending with no IPs,
creationTimestamp = S - 60 s, NodeIP 196.168.0.1, CIDR 10.0.0.1/8.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import abi

S0 = 1704067200  # 2024-01-01T00:00:00Z
NODE_IP = "196.168.0.1"
CIDR = "10.0.0.1/8"
PODS_PER_NODE = 10
BUCKETS = 4096


def node_names(first: int, count: int) -> np.ndarray:
    """`node-%07d` names as a (count, 12) uint8 array."""
    idx = np.arange(first, first + count, dtype=np.int64)
    out = np.empty((count, 12), np.uint8)
    out[:, :5] = np.frombuffer(b"node-", np.uint8)
    for k in range(7):
        out[:, 11 - k] = ord("0") + (idx // 10 ** k) % 10
    return out


def fnv1a32_rows(rows: np.ndarray) -> np.ndarray:
    h = np.full(rows.shape[0], 0x811C9DC5, np.uint32)
    prime = np.uint32(0x01000193)
    with np.errstate(over="ignore"):
        for k in range(rows.shape[1]):
            h = (h ^ rows[:, k].astype(np.uint32)) * prime
    return h


def slots_for(total_nodes: int, buckets: int = BUCKETS, pods_per_node: int = PODS_PER_NODE):
    """Per-bucket slot capacities with ~7 sigma headroom over the Poisson load."""
    avg = total_nodes / buckets
    cn = int(math.ceil(avg + 7 * math.sqrt(max(avg, 1.0)) + 4))
    cn = (cn + 3) // 4 * 4
    cp = (cn * pods_per_node + 7) // 8 * 8
    return cn, cp


@dataclass
class Fleet:
    total_nodes: int
    rank: int
    world: int
    names: np.ndarray        # (n_local, 12) names owned by this rank
    node_events: np.ndarray  # NODE_EVENT_DTYPE
    arena: bytes
    cn: int
    cp: int


def make_fleet(nodes_per_rank: int, rank: int = 0, world: int = 1, buckets: int = BUCKETS) -> Fleet:
    """Weak scaling: the fleet has nodes_per_rank * world nodes; this rank owns
    the nodes whose bucket falls in its contiguous bucket range."""
    total = nodes_per_rank * world
    names = node_names(0, total)
    b = fnv1a32_rows(names) & np.uint32(buckets - 1)
    lo = rank * buckets // world
    hi = (rank + 1) * buckets // world
    mine = names[(b >= lo) & (b < hi)]
    n = mine.shape[0]
    ev = np.zeros(n, abi.NODE_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["managed"] = 1
    ev["lockable"] = 1
    ev["name"]["off"] = np.arange(n, dtype=np.uint32) * 12
    ev["name"]["len"] = 12
    cn, cp = slots_for(total, buckets)
    return Fleet(total, rank, world, mine, ev, mine.tobytes(), cn, cp)


def pod_events(node_handles: np.ndarray, spec_id: int, pods_per_node: int = PODS_PER_NODE,
               creation: int = S0 - 60) -> np.ndarray:
    """Pending pods (status {phase: Pending}, no IPs), pods_per_node per node."""
    n = node_handles.shape[0] * pods_per_node
    ev = np.zeros(n, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    ev["handle"] = -1
    ev["spec_id"] = spec_id
    ev["node_handle"] = np.repeat(node_handles.astype(np.int32), pods_per_node)
    ev["creation_unix"] = creation
    return ev


def build_engine_fleet(engine_cls, nodes_per_rank, rank=0, world=1, device=0, cidr=CIDR, node_ip=NODE_IP,
                       start=S0, buckets=BUCKETS, pods_per_node=PODS_PER_NODE, **cfg_kw):
    """Create an engine (or oracle) for this rank and ingest its share of the
    fleet.  Returns (engine, fleet, pod_handles)."""
    from .engine import make_config
    fl = make_fleet(nodes_per_rank, rank, world, buckets)
    cfg = make_config(cidr=cidr, node_ip=node_ip, start_time=start, buckets=buckets,
                      node_slots_per_bucket=fl.cn, pod_slots_per_bucket=fl.cp, rank=rank, world_size=world,
                      device=device, **cfg_kw)
    e = engine_cls(cfg)
    spec = e.register_pod_spec([("fake-pod", "fake")])
    hs, st = e.ingest_nodes_raw(fl.node_events, fl.arena)
    if (st != 0).any():
        raise RuntimeError("node ingest rejected %d records (first code %d)" % ((st != 0).sum(), st[st != 0][0]))
    pods = pod_events(hs, spec, pods_per_node)
    ph, pst, _ = e.ingest_pods_raw(pods, b"")
    if (pst != 0).any():
        raise RuntimeError("pod ingest rejected %d records (first code %d)" % ((pst != 0).sum(), pst[pst != 0][0]))
    return e, fl, ph
