"""Shared multi-rank scenario (world_size >= 2) for the gloo CPU test (oracle
shards) and the single-GPU two-process engine test.  Every rank receives the
whole event stream, keeps what it owns (KWOK_ENOTMINE for the rest), forwards
ingest-time releases to the other ranks (kwok_pool_put), and exchanges
per-tick pool/counter data through the allgather hook."""
from __future__ import annotations

import ctypes as C
import os
import socket

import numpy as np

from kwok_amd import abi
from kwok_amd.engine import make_config

BUCKETS, CN, CP = 64, 32, 512
CIDR = "10.0.0.1/20"
BIG_CIDR = "10.0.0.1/16"  # the "big" scenario: > 2048 releases per rank in one tick (exchange lists not inline)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def gloo_allgather_fn():
    """kwok_allgather_fn over torch.distributed (gloo, host memory)."""
    import torch
    import torch.distributed as dist

    def fn(user, send, nbytes, recv):
        try:
            w = dist.get_world_size()
            src = torch.frombuffer(bytearray(C.string_at(send, nbytes)), dtype=torch.uint8)
            outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(w)]
            dist.all_gather(outs, src)
            buf = torch.cat(outs).numpy()  # keep alive across the copy
            C.memmove(recv, buf.ctypes.data, nbytes * w)
            return 0
        except Exception as ex:  # noqa: BLE001
            print("allgather failed:", ex)
            return 1
    return fn


def make(cls, rank, world, allgather=None, device=0, big=False, comm_id=None):
    cfg = make_config(cidr=BIG_CIDR if big else CIDR, node_ip="196.168.0.1", buckets=BUCKETS, node_slots_per_bucket=CN,
                      pod_slots_per_bucket=CP, rank=rank, world_size=world, device=device, allgather=allgather,
                      comm_id=comm_id)
    return cls(cfg)


def scenario(seed=11, ticks=5, big=False, foreign_from=0):
    """A deterministic list of per-tick event batches (dict form).  big: 12000
    pods, then 6000 deletions in one tick (every rank's release list is longer
    than the inline exchange message holds).  foreign_from: pods are created
    with podIPs of their own (3%, possibly another pod's address) only from
    that tick on: the ticks before it run quiet (Use checks skipped) on every
    rank, and the first foreign address ends that on every rank."""
    rng = np.random.default_rng(seed)
    names = ["node-%07d" % i for i in range(400)]
    out = []
    pid = 0
    live = []
    for t in range(ticks):
        nodes, pods = [], []
        if t == 0:
            for n in names:
                nodes.append(dict(op="upsert", name=n, managed=bool(rng.random() < 0.9),
                                  lockable=bool(rng.random() < 0.95)))
            k = 12000 if big else 3000
        else:
            k = 400
            for n in rng.choice(names, 4, replace=False):  # flaps
                nodes.append(dict(op="delete", name=str(n)))
                nodes.append(dict(op="upsert", name=str(n), managed=True, lockable=True))
            ndel = 6000 if big and t == 2 else 300
            for i in rng.choice(len(live), min(len(live), ndel), replace=False):
                pods.append(dict(op="deleting", key=live[i], fin=bool(rng.random() < 0.5)))
            for i in rng.choice(len(live), 60, replace=False):
                pods.append(dict(op="ext_delete", key=live[i]))
        for _ in range(k):
            key = "pod-%06d" % pid
            pid += 1
            ip = "10.0.%d.%d" % (rng.integers(0, 4), rng.integers(1, 255)) if rng.random() < 0.03 else ""
            ip = ip if t >= foreign_from else ""
            pods.append(dict(op="new", key=key, node=str(rng.choice(names)), ip=ip,
                             phase=int(rng.choice([abi.PHASE_PENDING, abi.PHASE_PENDING, abi.PHASE_NONE])),
                             fin=bool(rng.random() < 0.3)))
            live.append(key)
        gone = {p["key"] for p in pods if p["op"] in ("deleting", "ext_delete")}
        live = [k for k in live if k not in gone]
        out.append((nodes, pods))
    return out


class Runner:
    """Feeds the scenario to one backend (a shard or the whole fleet)."""

    def __init__(self, backend, world=1, rank=0, exchange_puts=None):
        self.b = backend
        self.world, self.rank = world, rank
        self.exchange_puts = exchange_puts
        self.spec = backend.register_pod_spec([("fake-pod", "fake")])
        self.handles = {}  # pod key -> handle (owned pods only)
        self.state = {}    # pod key -> (phase, hostip, podip) as last seen
        self.now = 1704067230

    def run_tick(self, nodes, pods, pair=False):
        if nodes:
            ar = abi.Arena()
            ev = np.zeros(len(nodes), abi.NODE_EVENT_DTYPE)
            for i, n in enumerate(nodes):
                ev[i]["op"] = abi.OP_DELETE if n["op"] == "delete" else abi.OP_UPSERT
                ev[i]["name"] = ar.ref(n["name"])
                ev[i]["managed"] = 1 if n.get("managed") else 0
                ev[i]["lockable"] = 1 if n.get("lockable") else 0
            _, st = self.b.ingest_nodes_raw(ev, bytes(ar.buf))
            assert set(st.tolist()) <= {abi.OK, abi.ENOTMINE, abi.ENOTFOUND}, st
        released = []
        for p in pods:  # one record per call keeps the key -> handle bookkeeping simple
            ar = abi.Arena()
            ev = np.zeros(1, abi.POD_EVENT_DTYPE)
            r = ev[0]
            r["spec_id"] = self.spec
            r["node_handle"] = -1
            r["creation_unix"] = 1704067140
            if p["op"] == "new":
                r["op"] = abi.OP_UPSERT
                r["handle"] = -1
                r["node_name"] = ar.ref(p["node"])
                r["phase"] = p["phase"]
                fl = abi.POD_STATUS_NONEMPTY if p["phase"] == abi.PHASE_PENDING or p["ip"] else 0
                fl |= abi.POD_HAS_FINALIZERS if p["fin"] else 0
                r["flags"] = fl
                r["pod_ip"] = ar.ref(p["ip"])
            else:
                h = self.handles.get(p["key"])
                if h is None:
                    continue  # another rank's pod
                cur = self.state_of(h)
                r["handle"] = h
                if cur["podip"]:
                    r["pod_ip"] = ar.ref(cur["podip"])
                if cur["hostip"]:
                    r["host_ip"] = ar.ref(cur["hostip"])
                r["phase"] = cur["phase"]
                if p["op"] == "deleting":
                    r["op"] = abi.OP_UPSERT
                    fl = abi.POD_DELETING | (abi.POD_HAS_FINALIZERS if p["fin"] else 0)
                    if cur["phase"] == abi.PHASE_RUNNING:
                        fl |= abi.POD_CONFORMS | abi.POD_STATUS_NONEMPTY
                    elif cur["phase"] == abi.PHASE_PENDING or cur["podip"]:
                        fl |= abi.POD_STATUS_NONEMPTY
                    r["flags"] = fl
                else:
                    r["op"] = abi.OP_DELETE
            hs, st, rel = self.b.ingest_pods_raw(ev, bytes(ar.buf))
            if st[0] == abi.OK and p["op"] == "new":
                self.handles[p["key"]] = int(hs[0])
            elif st[0] == abi.OK and p["op"] == "ext_delete":
                del self.handles[p["key"]]
            else:
                assert st[0] in (abi.OK, abi.ENOTMINE), (p, st[0])
            if rel[0]:
                released.append(int(rel[0]))
        if self.exchange_puts is not None:
            others = self.exchange_puts(released)
            if others:
                self.b.pool_put(np.array(others, np.uint32))
        if not pair:
            return self._done(self.b.tick(self.now))
        # two ticks with no events between: queued back to back where the backend
        # can (kwok_tick_submit / _collect), one after the other otherwise
        if hasattr(self.b, "tick_submit"):
            self.b.tick_submit(self.now)
            self.b.tick_submit(self.now + 30)
            first = self._done(self.b.tick_collect())
            return [first, self._done(self.b.tick_collect())]
        first = self._done(self.b.tick(self.now))
        return [first, self._done(self.b.tick(self.now))]

    def _done(self, out):
        self.now += 30
        for h, _ in out.deletes:
            for k in [k for k, v in self.handles.items() if v == h]:
                del self.handles[k]
        return out

    def state_of(self, h):
        used, phase, hip, pip = self.b.dump_pods(h, 1)
        return dict(phase=int(phase[0]), hostip=abi.ip4s(int(hip[0])), podip=abi.ip4s(int(pip[0])))


def run_all(runner, sc, pair=False):
    """Summaries of every tick of scenario sc (pair: each step is two ticks,
    queued back to back on backends that can)."""
    out = []
    trace = os.environ.get("KWOK_TEST_TRACE")
    for t, (n, p) in enumerate(sc):
        if trace:
            print("[run_all] rank %d tick %d: %d node, %d pod records" % (runner.rank, t, len(n), len(p)), flush=True)
        r = runner.run_tick(n, p, pair=pair)
        out += [summarize(x) for x in (r if pair else [r])]
    return out


def summarize(out):
    """Order-preserving, comparable view of one tick's outputs."""
    hb = out.heartbeat_body(0) if len(out.heartbeat_nodes) else b""
    return dict(hb=[int(h) for h in out.heartbeat_nodes], hb_body=hb,
                inits=[(int(h), b) for h, b in out.node_inits],
                pods=[(int(h), b) for h, b in out.pod_patches],
                deletes=[tuple(d) for d in out.deletes], counters=dict(out.counters))
