"""Shared helpers of the GPU parity tests: the HIP engine and the CPU oracle
driven with the same event batches, compared output by output (handles, patch
bytes, deletes, counters) and on the full pod state."""
import numpy as np
from numpy.lib.stride_tricks import as_strided

from kwok_amd import abi
from kwok_amd.engine import Engine, make_config
from oracle.oracle import Oracle


def compare(e_out, o_out, where):
    assert list(e_out.heartbeat_nodes) == list(o_out.heartbeat_nodes), where + " heartbeat handles"
    n = len(e_out.heartbeat_nodes)
    if n:
        hb = o_out.heartbeat_body(0)
        a = np.frombuffer(e_out.arena, np.uint8)[e_out.heartbeat_off:e_out.heartbeat_off + n * e_out.heartbeat_stride]
        a = a.reshape(n, e_out.heartbeat_stride)[:, :e_out.heartbeat_len]
        ok = (a == np.frombuffer(hb, np.uint8)[None, :])
        if not ok.all():
            bad = np.nonzero(~ok.all(axis=1))[0]
            pos = np.nonzero(~ok[bad[0]])[0]
            raise AssertionError("%s heartbeat bytes: %d of %d bodies differ (first #%d at bytes %s); got %r want %r" % (
                where, len(bad), n, bad[0], list(pos[:8]), bytes(a[bad[0]][pos[0]:pos[0] + 24]), hb[pos[0]:pos[0] + 24]))
        ob = np.frombuffer(o_out.arena, np.uint8)[o_out.heartbeat_off:o_out.heartbeat_off + n * len(hb)]
        assert (ob.reshape(n, len(hb)) == np.frombuffer(hb, np.uint8)[None, :]).all()
    assert [h for h, _ in e_out.node_inits] == [h for h, _ in o_out.node_inits], where + " node-init handles"
    assert [b for _, b in e_out.node_inits] == [b for _, b in o_out.node_inits], where + " node-init bytes"
    assert [h for h, _ in e_out.pod_patches] == [h for h, _ in o_out.pod_patches], where + " pod-patch handles"
    bad = [h for (h, b), (_, c) in zip(e_out.pod_patches, o_out.pod_patches) if b != c]
    assert not bad, where + " pod-patch bytes differ for %d pods, first %d" % (len(bad), bad[0])
    assert e_out.deletes == o_out.deletes, where + " deletes"
    assert e_out.counters == o_out.counters, where + " counters"


def compare_state(e, o, n_slots, where):
    eu, ep, eh, ei = e.dump_pods(0, n_slots)
    ou, op, oh, oi = o.dump_pods(0, n_slots)
    assert (eu == ou).all(), where + " pod slots"
    assert (ep == op).all(), where + " phases"
    assert (eh == oh).all(), where + " hostIPs"
    assert (ei == oi).all(), where + " podIPs"


class Driver:
    """Applies the same random event batches to engine and oracle."""

    DEFAULT_SPECS = [([("fake-pod", "fake")], [], []),
                     ([("a", "img-a"), ("b", "img/b:v2")], [("init", "busybox")], ["g.io/x"])]

    def __init__(self, cfg_kw, seed, specs=None):
        self.e = Engine(make_config(**cfg_kw))
        self.o = Oracle(make_config(**cfg_kw))
        self.rng = np.random.default_rng(seed)
        self.cfg = cfg_kw
        self.spec = [self.e.register_pod_spec(*sp) for sp in (specs or self.DEFAULT_SPECS)]
        assert self.spec == [self.o.register_pod_spec(*sp) for sp in (specs or self.DEFAULT_SPECS)]
        self.n_slots = cfg_kw["buckets"] * (cfg_kw.get("pod_handle_stride") or cfg_kw["pod_slots_per_bucket"])
        self.spec_of = np.zeros(self.n_slots, np.int32)   # immutable pod fields, by handle
        self.ctime_of = np.zeros(self.n_slots, np.int64)
        self.now = 1704067230

    def nodes(self, names, managed, lockable, op=abi.OP_UPSERT, phase=abi.PHASE_NONE, status=None):
        """status: optional per-node dicts {addresses, allocatable, capacity (JSON
        strings), nodeInfo {key: value}} as the codec would decode them"""
        ar = abi.Arena()
        ev = np.zeros(len(names), abi.NODE_EVENT_DTYPE)
        ev["op"] = op
        ev["managed"] = managed
        ev["lockable"] = lockable
        ev["phase"] = phase
        for i, n in enumerate(names):
            ev[i]["name"] = ar.ref(n)
            if status is not None and status[i]:
                st = status[i]
                for f in ("addresses", "allocatable", "capacity"):
                    ev[i][f] = ar.ref(st.get(f, ""))
                for k, key in enumerate(abi.NODEINFO_KEYS):
                    ev[i]["node_info"][k] = ar.ref(st.get("nodeInfo", {}).get(key, ""))
        a = bytes(ar.buf)
        h1, s1 = self.e.ingest_nodes_raw(ev, a)
        h2, s2 = self.o.ingest_nodes_raw(ev, a)
        assert (h1 == h2).all() and (s1 == s2).all()
        return h1, s1

    def pods(self, ev, arena=b""):
        h1, s1, r1 = self.e.ingest_pods_raw(ev, arena)
        h2, s2, r2 = self.o.ingest_pods_raw(ev, arena)
        assert (h1 == h2).all() and (s1 == s2).all() and (r1 == r2).all()
        new = (ev["op"] == abi.OP_UPSERT) & (ev["handle"] < 0) & (s1 == 0)
        self.spec_of[h1[new]] = ev["spec_id"][new]
        self.ctime_of[h1[new]] = ev["creation_unix"][new]
        return h1, s1, r1

    def tick(self, where):
        eo, oo = self.e.tick(self.now), self.o.tick(self.now)
        self.now += 30
        compare(eo, oo, where)
        compare_state(self.e, self.o, self.n_slots, where)
        return eo

    def tick_pair(self, where):
        """two ticks queued back to back on the engine, one after the other on the oracle"""
        self.e.tick_submit(self.now)
        self.e.tick_submit(self.now + 30)
        for k in range(2):
            eo, oo = self.e.tick_collect(), self.o.tick(self.now)
            self.now += 30
            compare(eo, oo, "%s (queued %d)" % (where, k))
        compare_state(self.e, self.o, self.n_slots, where)

    def live(self):
        used, phase, hip, pip = self.o.dump_pods(0, self.n_slots)
        idx = np.nonzero(used)[0]
        return idx, phase[idx], hip[idx], pip[idx]


def new_pods(rng, node_handles, n, spec_ids, with_ip_frac=0.0, ip_range=None, host_ips=(), host_ip_frac=0.0,
             years=0):
    """Pending / empty-status pods on random nodes; optionally with existing
    podIPs from ip_range, existing hostIPs drawn from host_ips, and creation
    times spread over `years` years (timestamp formatting)."""
    ev = np.zeros(n, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1
    ev["node_handle"] = rng.choice(node_handles, n)
    ev["spec_id"] = rng.choice(spec_ids, n)
    ev["creation_unix"] = 1704067200 - rng.integers(0, max(10 ** 6, years * 31_557_600), n)
    ph = rng.choice([abi.PHASE_PENDING, abi.PHASE_PENDING, abi.PHASE_NONE], n)
    ev["phase"] = ph
    fl = np.where(ph == abi.PHASE_PENDING, abi.POD_STATUS_NONEMPTY, 0)
    fl |= np.where(rng.random(n) < 0.3, abi.POD_HAS_FINALIZERS, 0)
    fl |= np.where(rng.random(n) < 0.03, abi.POD_DISREGARD, 0)
    ev["flags"] = fl
    arena = b""
    if (with_ip_frac and ip_range) or (host_ip_frac and host_ips):
        ar = abi.Arena()
        if with_ip_frac and ip_range:
            lo, hi = ip_range
            for i in np.nonzero(rng.random(n) < with_ip_frac)[0]:
                ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(rng.integers(lo, hi))))
                ev[i]["flags"] |= abi.POD_STATUS_NONEMPTY
        if host_ip_frac and host_ips:
            for i in np.nonzero(rng.random(n) < host_ip_frac)[0]:
                ev[i]["host_ip"] = ar.ref(host_ips[int(rng.integers(0, len(host_ips)))])
                ev[i]["flags"] |= abi.POD_STATUS_NONEMPTY
        arena = bytes(ar.buf)
    return ev, arena


def mark_deleting(rng, d, handles):
    """Modified events with a deletionTimestamp for existing pods (state kept)."""
    idx, phase, hip, pip = d.live()
    pos = np.searchsorted(idx, handles)
    ar = abi.Arena()
    ev = np.zeros(len(handles), abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = handles
    ev["node_handle"] = -1
    ev["spec_id"] = d.spec_of[handles]
    ev["phase"] = phase[pos]
    ev["creation_unix"] = d.ctime_of[handles]
    fl = abi.POD_DELETING | np.where(rng.random(len(handles)) < 0.5, abi.POD_HAS_FINALIZERS, 0)
    fl |= np.where(phase[pos] == abi.PHASE_RUNNING, abi.POD_CONFORMS | abi.POD_STATUS_NONEMPTY, 0)
    ev["flags"] = fl
    for i in range(len(handles)):
        if hip[pos[i]]:
            ev[i]["host_ip"] = ar.ref(abi.ip4s(int(hip[pos[i]])))
        if pip[pos[i]]:
            ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(pip[pos[i]])))
    return ev, bytes(ar.buf)


def external_deletes(d, handles):
    idx, phase, hip, pip = d.live()
    pos = np.searchsorted(idx, handles)
    ar = abi.Arena()
    ev = np.zeros(len(handles), abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_DELETE
    ev["handle"] = handles
    for i in range(len(handles)):
        if pip[pos[i]]:
            ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(pip[pos[i]])))
    return ev, bytes(ar.buf)


# ---- vectorised comparison for fleets of millions of objects ----------------
def rows(arena, off, length):
    """arena[off[i] : off[i] + length] for every i, as one (n, length) array"""
    v = as_strided(arena, (arena.size - length + 1, length), (1, 1))
    return v[off.astype(np.int64)]


def compare_patches(ea, eo, el, oa, oo, ol, what):
    assert (el == ol).all(), what + " lengths"
    for L in np.unique(el):
        sel = np.nonzero(el == L)[0]
        for part in np.array_split(sel, max(1, len(sel) // 1_000_000)):
            a, b = rows(ea, eo[part], int(L)), rows(oa, oo[part], int(L))
            bad = np.nonzero((a != b).any(axis=1))[0]
            assert len(bad) == 0, "%s: %d patches of length %d differ, first at #%d" % (what, len(bad), L, part[bad[0]])


def patch_digests(arena, off, length):
    """A 64-bit digest per patch (a random linear form of its bytes, the same
    weights in every process): compares patch bytes across processes without
    moving them."""
    out = np.zeros(len(off), np.uint64)
    length = np.asarray(length)
    for L in np.unique(length):
        sel = np.nonzero(length == L)[0]
        w = np.random.default_rng(int(L)).integers(1, 1 << 62, int(L), dtype=np.uint64) | np.uint64(1)
        for part in np.array_split(sel, max(1, len(sel) // 50_000)):
            r = rows(arena, np.asarray(off)[part], int(L)).astype(np.uint64)
            out[part] = (r * w[None, :]).sum(axis=1, dtype=np.uint64)
    return out


def shim_read_check(e, O, res, chunk=64 << 20):
    """The Go drop-in's read sequence (integration/go/.../engine_cgo.go tick /
    applyPatches), replayed through ctypes on the engine's collected tick and
    checked byte for byte against the oracle's outputs O (read_arrays):
    kwok_read_outputs without an arena (the lists), kwok_read_arena of ONE
    heartbeat body, then the node-init and pod patches in pieces of at most
    `chunk` bytes, 64-bit offsets.  Returns (pieces, bytes read)."""
    import ctypes as C
    n = {k: getattr(res, k) for k in ("n_heartbeat", "n_node_init", "n_pod_patch", "n_delete")}
    L = {"hb": np.empty(n["n_heartbeat"], np.int32),
         "ini": np.empty(n["n_node_init"], np.int32), "ini_off": np.empty(n["n_node_init"], np.uint64),
         "ini_len": np.empty(n["n_node_init"], np.uint32),
         "pp": np.empty(n["n_pod_patch"], np.int32), "pp_off": np.empty(n["n_pod_patch"], np.uint64),
         "pp_len": np.empty(n["n_pod_patch"], np.uint32),
         "dl": np.empty(n["n_delete"], np.int32), "dlf": np.empty(n["n_delete"], np.uint8)}
    p = lambda k: L[k].ctypes.data if L[k].size else None  # noqa: E731
    out = abi.Outputs(p("hb"), 0, p("ini"), p("ini_off"), p("ini_len"), p("pp"), p("pp_off"), p("pp_len"),
                      p("dl"), p("dlf"), None, 0, 0)
    e._check(e._fn("read_outputs")(e._h, C.byref(out)), "read_outputs (lists only)")
    assert out.arena_copied == 0
    for a, b in (("hb", "heartbeat_nodes"), ("ini", "node_init_nodes"), ("pp", "pod_patch_pods"),
                 ("dl", "delete_pods"), ("dlf", "delete_has_finalizers")):
        assert (L[a] == O[b]).all(), b
    total = pieces = 0
    if n["n_heartbeat"]:
        body = e.read_arena(out.heartbeat_off, res.heartbeat_len)
        total += body.size
        assert (body == O["arena"][O["heartbeat_off"]:O["heartbeat_off"] + O["heartbeat_len"]]).all(), "heartbeat body"
    for hs, offs, lens, oo, ol, what in ((L["ini"], L["ini_off"], L["ini_len"], O["node_init_off"], O["node_init_len"],
                                         "node inits"),
                                        (L["pp"], L["pp_off"], L["pp_len"], O["pod_patch_off"], O["pod_patch_len"],
                                         "pod patches")):
        ends = offs.astype(np.int64) + lens
        assert (np.diff(offs.astype(np.int64)) > 0).all(), what + ": offsets increase"
        i = 0
        while i < len(hs):
            lo = int(offs[i])
            j = max(i + 1, int(np.searchsorted(ends, lo + chunk, side="right")))  # the shim's greedy piece
            buf = e.read_arena(lo, int(ends[j - 1]) - lo)
            assert buf.size <= chunk or j == i + 1
            compare_patches(buf, offs[i:j] - np.uint64(lo), lens[i:j], O["arena"], oo[i:j], ol[i:j], what)
            total += buf.size
            pieces += 1
            i = j
    return pieces, total


def compare_tick(e, o, where, once=False):
    """once: a heartbeat-once engine, whose arena holds the one heartbeat body"""
    E, O = e.read_arrays(heartbeat_once=once) if once else e.read_arrays(), o.read_arrays()
    assert E["counters"] == O["counters"], where
    assert (E["heartbeat_nodes"] == O["heartbeat_nodes"]).all(), where + " heartbeat handles"
    n = len(E["heartbeat_nodes"])
    if n and once:
        body = O["arena"][O["heartbeat_off"]:O["heartbeat_off"] + O["heartbeat_len"]]
        assert (E["arena"][E["heartbeat_off"]:E["heartbeat_off"] + E["heartbeat_len"]] == body).all(), where
    elif n:
        body = O["arena"][O["heartbeat_off"]:O["heartbeat_off"] + O["heartbeat_len"]]
        hb = E["arena"][E["heartbeat_off"]:E["heartbeat_off"] + n * E["heartbeat_stride"]]
        hb = hb.reshape(n, E["heartbeat_stride"])[:, :E["heartbeat_len"]]
        assert (hb == body[None, :]).all(), where + " heartbeat bodies"
    for k in ("node_init_nodes", "pod_patch_pods", "delete_pods", "delete_has_finalizers"):
        assert (E[k] == O[k]).all(), where + " " + k
    compare_patches(E["arena"], E["node_init_off"], E["node_init_len"], O["arena"], O["node_init_off"],
                    O["node_init_len"], where + " node inits")
    compare_patches(E["arena"], E["pod_patch_off"], E["pod_patch_len"], O["arena"], O["pod_patch_off"],
                    O["pod_patch_len"], where + " pod patches")
    return E["counters"]
