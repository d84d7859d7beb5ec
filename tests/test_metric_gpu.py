"""GPU parity at the metric's own configuration (BASELINE.json metric "at 1M
nodes/10M pods", north_star "1M simulated nodes / 10M pods stepped per tick"):
1M nodes x 10M pods on one MI355X against the CPU restatement (its OpenMP
sweeps), byte for byte on the initial tick (1M node-init patches, 10M
Pending->Running patches with IP allocation) and on a steady tick (1M
heartbeats), plus size-independent properties of the allocation.  The
comparison is vectorised (numpy views over both arenas): the per-patch
Python objects of the small-trace tests would not fit."""
import ipaddress

import numpy as np
import pytest
from gpu_common import compare_tick, shim_read_check
from kwok_amd import workload
from kwok_amd.engine import Engine
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

NODES = 1_000_000


@pytest.mark.timeout(900)
def test_metric_config_1m_nodes_10m_pods():
    e, fl, ph = workload.build_engine_fleet(Engine, NODES)
    o, _, ph2 = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=0), NODES)
    assert (ph == ph2).all() and len(ph) == 10 * NODES
    n_slots = workload.BUCKETS * fl.cp
    r0 = e.tick(workload.S0 + 30, read=False)
    o.tick(workload.S0 + 30, read=False)
    c = compare_tick(e, o, "1M tick 0")
    assert c["pod_patch"] == 10 * NODES and c["node_init"] == NODES and c["alloc"] == 10 * NODES
    # the Go drop-in's hand-off (lists, one heartbeat body, the ~7 GB of patches in
    # 64 MiB pieces through kwok_read_arena): every byte against the oracle
    assert r0.arena_bytes > 1 << 32
    pieces, nbytes = shim_read_check(e, o.read_arrays(), r0)
    assert pieces > 64 and nbytes > 1 << 32, (pieces, nbytes)
    used, phase, hip, pip = e.dump_pods(0, n_slots)
    live = used.astype(bool)
    ips = pip[live]
    base = int(ipaddress.IPv4Address("10.0.0.1"))
    # ipPool.new hands out base, base+1, ... in canonical (bucket, slot) order (utils.go:68-81)
    assert (ips == base + np.arange(10 * NODES, dtype=np.uint32)).all()
    assert (phase[live] == 2).all() and (hip[live] == int(ipaddress.IPv4Address("196.168.0.1"))).all()
    ou, op, oh, oi = o.dump_pods(0, n_slots)
    assert (ou == used).all() and (op == phase).all() and (oh == hip).all() and (oi == pip).all()
    # a steady tick: 1M identical heartbeats, every pod re-checked, nothing patched
    e.tick(workload.S0 + 60, read=False)
    o.tick(workload.S0 + 60, read=False)
    c = compare_tick(e, o, "1M tick 1")
    assert c["heartbeat"] == NODES and c["pod_patch"] == 0 and c["evaluated"] == 10 * NODES
    e.close()
    o.close()
