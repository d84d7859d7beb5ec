#!/usr/bin/env python3
"""bench.py - kwok fake-kubelet tick on MI355X (BASELINE.json metric:
"state transitions/sec at 1M nodes/10M pods, 1-8 MI355X; % HBM roofline").

Workload (N=1): the metric's configuration - 1M nodes x 10M pods (10 pods per
node, the reference benchmark's pod shape) stepped per tick on one MI355X:
steady-state heartbeat + status ticks (BASELINE configs[1]'s tick at the
metric's size).  Weak scaling: every rank owns 1M nodes / 10M pods of a fleet
of N x 1M nodes hashed into 4096 buckets (contiguous bucket ranges per rank);
ranks exchange pool / counter data over RCCL every tick.  The CIDR is
10.0.0.1/8 (/4 once the fleet has more than 16M pods) so that every fresh IP
lies in the CIDR.

A step = one tick (one heartbeat interval at a fixed clock): the heartbeat patch
of every managed node, the lock check of every node, the re-evaluation of
every pod, ipPool bookkeeping and the host collecting the tick's result, with
all state resident in HBM.  Steps are queued (kwok_tick_submit for tick k+1
before kwok_tick_collect of tick k).  Reported beside `value`:
  * the same steps one blocking kwok_tick each;
  * the same steps with the per-tick hand-off a Go caller consumes
    (kwok_read_outputs, KWOK_READ_HEARTBEAT_ONCE: one heartbeat body + the
    patch region + the delete list; the heartbeat handle list only when its
    epoch changes) - PCIe-inclusive;
  * the initial tick (1M node-init patches + 10M Pending->Running patches with
    IP allocation), timed on its own, with its own roofline (k_emit).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# torch's wheel bundles its own HIP runtime (loaded by file name).  Initialise
# it first so that libkwok_engine.so binds the SAME runtime (its NEEDED
# sonames resolve to the already-loaded copies): one runtime per process, and
# torch.cuda.synchronize() covers the engine's stream.
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# KWOK_BENCH_REHEARSAL=1: every rank on GPU 0 and the exchange over the host
# allgather hook (gloo) instead of RCCL - rehearses the N>1 bench on a one-GPU
# box (RCCL refuses two ranks on one GPU); never used for reported numbers
REHEARSAL = os.environ.get("KWOK_BENCH_REHEARSAL") == "1"
torch.cuda.set_device(0 if REHEARSAL else int(os.environ.get("LOCAL_RANK", "0")))

from kwok_amd import abi  # noqa: E402
from kwok_amd import engine as keng  # noqa: E402
from kwok_amd import workload  # noqa: E402

keng.load_engine_lib()

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
NODES_PER_RANK = 1_000_000
# algorithmic HBM bytes (SURVEY.md §8(d) byte model):
#   steady tick, per managed node: heartbeat 1 B flags + 4 B hb-time + 4 B
#   out-index + the 1059-byte patch = 1068 B, plus a no-op re-lock check 9 B;
#   per live pod a no-op re-check 10 B
NODE_BYTES = 1068 + 9
POD_BYTES = 10
NODE_STATE_BYTES = 9 + 9   # the same without the materialised patch (state-only line)
NODE_SLOT_BYTES = 1          # k_once: a node's state byte
#   initial tick, per node init 1471 B (9 B check + 4 B index + 1458 B patch), per
#   Pending->Running pod 577 B (10 + 4 + 8 B reads, 1 + 4 + 4 B writes, ~542 B patch)
INIT_BYTES = 1471
POD_PATCH_BYTES = 577
#   C4 tick, per deleted pod: 10 B re-check + 4 B handle + 1 B finalizer flag + 4 B release
DELETE_BYTES = 19
CHURN_WARMUP = 2  # untimed churn batches before the timed steps (see churn_leg)
PMC_FILE = "r12_pmc.json"
ONCE_PMC_FILE = "r12_once_pmc.json"  # the heartbeat-once leg's k_once (tools/gpu_full.sh)
C4_PMC_FILE = "r12_c4once_pmc.json"  # the heartbeat-once engine's C4 tick kernels (tools/gpu_c4once.sh)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nodes-per-rank", type=int, default=NODES_PER_RANK)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU restatement on rank 0 (N=1)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="threads of the all-core leg (0: all cores)")
    ap.add_argument("--cpu-ticks", type=int, default=5)
    ap.add_argument("--roofline-ticks", type=int, default=20)
    ap.add_argument("--churn-ticks", type=int, default=5, help="C4 churn ticks after the steady legs (N=1; 0: skip)")
    ap.add_argument("--flap-ticks", type=int, default=5, help="C5 flap ticks on a partially managed fleet (N=1; 0: skip)")
    ap.add_argument("--once-ticks", type=int, default=1, help="the KWOK_CFG_HEARTBEAT_ONCE legs (N=1; 0: skip)")
    ap.add_argument("--c2", type=int, default=1, help="BASELINE configs[1] at 100k x 1M (N=1; 0: skip)")
    ap.add_argument("--json-ticks", type=int, default=2, help="C4 from JSON documents, GPU codec (N=1; 0: skip)")
    ap.add_argument("--churn", type=int, default=0, help="pods churned per tick (0: nodes_per_rank, i.e. 1M at the "
                                                         "metric size: 2M create/delete per tick)")
    ap.add_argument("--emulate-ranks", type=int, default=8, help="N=1: a one-rank RCCL engine folding this many "
                                                                 "ranks' exchange messages (0: skip)")
    ap.add_argument("--leg", default="", help=argparse.SUPPRESS)  # (internal: one secondary leg, in a child process)
    ap.add_argument("--legs-inline", type=int, default=0,
                    help="run the secondary legs in this process instead of one child process each")
    return ap.parse_args()


SECONDARY_LEGS = ("flap", "flap_once", "hb_once", "c2", "emul")


def run_leg(name, a):
    """One secondary leg (N=1) of this process's arguments"""
    if name == "flap":
        return flap_leg(a.nodes_per_rank, a.flap_ticks)
    if name == "flap_once":
        return flap_leg(a.nodes_per_rank, a.flap_ticks, True)
    if name == "hb_once":
        return heartbeat_once_leg(a.nodes_per_rank, a.steps, a.warmup, a.churn_ticks, a.json_ticks)
    if name == "c2":
        return c2_leg(a.steps, a.warmup)
    if name == "emul":
        return emulated_ranks_leg(a.nodes_per_rank, a.emulate_ranks, 20, min(a.churn_ticks, 3))
    raise ValueError(name)


def leg(name, a):
    """A secondary leg in a child process of its own (the default): each leg's engine
    starts on a fresh device context, as a deployment's one engine per process does.
    Engines created one after another in one process measured slower ingest, ~0.1-0.2 ms
    per C4 batch by the third (tools/c4_seq_probe.py).  The child writes the leg's JSON
    on its stdout; its stderr is this process's."""
    if a.legs_inline:
        return run_leg(name, a)
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:] + ["--leg", name]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, timeout=900)
    if r.returncode != 0:
        raise RuntimeError("bench leg %s failed (exit %d)" % (name, r.returncode))
    return json.loads(r.stdout.decode().strip().splitlines()[-1])


def cidr_for(total_pods):
    return "10.0.0.1/8" if total_pods <= (1 << 24) - 16 else "10.0.0.1/4"


def transitions(c):
    # heartbeat + node init + pod patch + delete + release
    return c[0] + c[1] + c[2] + c[3] + c[5]


def oracle_steady(nodes, threads, ticks):
    """The C restatement (oracle/kwok_oracle.c, test infrastructure) on a fleet
    of `nodes` nodes x 10 pods: built and initial-ticked with all threads, then
    steady ticks on `threads` threads (its OpenMP sweeps) and on one thread.
    Returns ({threads: (transitions/s, ms per tick)}, cores, setup + initial s)."""
    from oracle.oracle import Oracle  # test infrastructure: baseline only
    t0 = time.perf_counter()
    o, _, _ = workload.build_engine_fleet(lambda cfg: Oracle(cfg, threads=threads), nodes,
                                          cidr=cidr_for(nodes * workload.PODS_PER_NODE))
    cores = o.threads
    o.tick(workload.S0 + 30, read=False)  # initial tick (locks + Pending->Running)
    t_init = time.perf_counter() - t0
    legs = {}
    now = workload.S0 + 60
    for th in (cores, 1):
        o.set_threads(th)
        trans = 0
        n = ticks if th > 1 else max(2, ticks // 2)
        t1 = time.perf_counter()
        for _ in range(n):
            r = o.tick(now, read=False)
            now += 30
            trans += transitions(r.counters)
        dt = time.perf_counter() - t1
        legs[th] = (trans / dt, dt / n * 1e3)
    o.close()
    return legs, cores, t_init


def cpu_baseline(nodes, threads, ticks):
    """The oracle timed on the GPU box's host cores: at the metric fleet (the
    baseline of `value`) and at BASELINE configs[0] (C1, 1k x 10k) and
    configs[1] (C2, 100k x 1M), each on all cores and on one"""
    legs, cores, t_init = oracle_steady(nodes, threads, ticks)
    cfgs = {}
    for label, n, k in (("C1", 1_000, 200), ("C2", 100_000, 2 * ticks)):
        lg, c, ti = oracle_steady(n, threads, k)
        cfgs[label] = {"nodes": n, "pods": n * workload.PODS_PER_NODE, "cores": c,
                       "value": lg[c][0], "ms_per_step": lg[c][1],
                       "single_core": {"value": lg[1][0], "ms_per_step": lg[1][1]}, "setup_initial_s": ti}
    return {"value": legs[cores][0], "unit": "transitions/s", "cores": cores, "kind": "port",
            "ms_per_step": legs[cores][1],
            "single_core": {"value": legs[1][0], "cores": 1, "ms_per_step": legs[1][1]},
            "configs": cfgs,
            "sample": "oracle/kwok_oracle.c (the C restatement, OpenMP sweeps), the same %d nodes x %d pods "
                      "fleet, steady ticks after the initial tick (setup + initial tick %.1fs on %d threads); "
                      "configs: C1 / C2 at their own sizes; the reference Go controllers cannot run here (no Go "
                      "toolchain)" % (nodes, nodes * workload.PODS_PER_NODE, t_init, cores)}


def churn_leg(e, fl, pod_handles, now, ticks, n_churn, rank=0, world=1, barrier=None, max_over_ranks=None,
              packed=12, ch=None, multi=False, once=False, together=False):
    """BASELINE configs[3] (C4) on the same fleet: per tick, n_churn pods marked
    for deletion (Modified events with their status, half with finalizers) and
    n_churn new Pending pods on the same nodes (workload.Churn).  A step =
    kwok_ingest_pods of that batch (2 x n_churn records, host threads + H2D +
    apply kernel) + one kwok_tick (1M deletes + releases, 1M Pending->Running
    patches reusing the released IPs).  Event generation (which reads the pod
    IPs back) sits between the timed steps.  CHURN_WARMUP untimed batches first.
    world > 1: every rank churns n_churn of its own pods per tick (weak
    scaling); the releases of all ranks cross the exchange (their lists are
    longer than the inline message: the second allgather), and each step is
    timed between barriers, max over ranks.  packed=12: the batch as
    kwok_pod_rec12 (12 B per record, kwok_ingest_pods_packed12: statuses as
    bytes, the creates' handles only, no release list at N=1); packed=20:
    kwok_pod_rec (20 B, kwok_ingest_pods_packed, every handle back); otherwise
    kwok_pod_event records with dotted-quad strings (48 B + strings).
    together (packed=12, one rank): kwok_ingest_pods_packed12_tick - the tick
    queued behind the batch's apply passes, collected after the call (ingest_ms:
    the call, tick_ms: kwok_tick_collect)."""
    barrier = barrier or torch.cuda.synchronize
    max_over_ranks = max_over_ranks or (lambda x: x)
    lo = rank * workload.BUCKETS // world
    hi = (rank + 1) * workload.BUCKETS // world
    n_handles = (hi - lo) * fl.cp
    # the batch and the per-record results live in page-locked host memory
    # (kwok_host_alloc): the ingest's copies to and from the GPU run by DMA
    if ch is None:  # (a later leg continues the previous leg's generator: its live pods)
        ch = workload.Churn(pod_handles, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, n_churn,
                            seed=7, first=lo * fl.cp, alloc=keng.host_array)
    ch.packed, ch.bufs = (packed if packed == 12 else bool(packed)), None
    if packed == 12:  # the creates' handles; multi rank: the releases too (kwok_pool_put material)
        outs = (keng.host_array((n_churn,), np.int32), keng.host_array((2 * n_churn,), np.int8),
                keng.host_array((2 * n_churn,), np.uint32) if world > 1 else None)
    elif packed:
        outs = (keng.host_array((2 * n_churn,), np.int32), keng.host_array((2 * n_churn,), np.int8),
                keng.host_array((2 * n_churn,), np.uint32) if world > 1 else None)
    else:
        outs = (keng.host_array((2 * n_churn,), np.int32), keng.host_array((2 * n_churn,), np.int32),
                keng.host_array((2 * n_churn,), np.uint32))
    dump = lambda: e.dump_pods(lo * fl.cp, n_handles)  # noqa: E731
    ing = tck = 0.0
    trans = recs = 0
    kern = emit = xch = 0.0
    phases = {}
    last = None
    steps = []
    # (the runtime's ~6 ms copy-engine queue creations, which used to land in one or two of a
    # process's first churn batches, now happen at engine create: profiles/r4v_sdma_ab.txt)
    warm = CHURN_WARMUP
    for k in range(ticks + warm + 1):
        ev, ar = ch.batch(dump, now)
        barrier()
        prof = k == ticks + warm  # one more step, profiled (HIP events), for the kernel times only
        if prof:
            e.profile_enable(True)
        t0 = time.perf_counter()
        if packed == 12:
            hs, st, _ = e.ingest_pods_packed12(ev, new_cap=len(ev) // 2, out=outs, tick_now=now if together else None)
        else:
            hs, st, _ = e.ingest_pods_packed(ev, out=outs) if packed else e.ingest_pods_raw(ev, ar, out=outs)
        t1 = time.perf_counter()
        r = e.tick_collect(read=False) if together else e.tick(now, read=False)
        t2 = time.perf_counter()
        if world > 1:
            barrier()
            t2 = time.perf_counter()
        ch.applied(hs.copy(), st, new_only=packed == 12)
        now += 30
        if prof:
            ph, nt = e.profile_read()
            e.profile_enable(False)
            kern, emit, xch = ph["kernel"] * ticks, ph["emit_kernel"] * ticks, ph["exchange"] * ticks
            phases = {k: v / max(nt, 1) for k, v in ph.items()}
        elif k >= warm:
            a, b = max_over_ranks(t1 - t0), max_over_ranks(t2 - t0)
            ing += a
            tck += b - a
            steps.append((a, b - a))
            trans += transitions(r.counters)
            recs += len(ev)
            last = dict(zip(abi.COUNTERS, list(r.counters)))
    return now, ch, {
        "workload": "C4 pod churn storm (BASELINE configs[3]) on the metric fleet: %d deletion-marked pods (50%% with "
                    "finalizers) + %d creates per tick%s" % (n_churn, n_churn, " per rank" if world > 1 else ""),
        "ticks": ticks, "records_per_tick": recs // max(ticks, 1) * world,
        "wire": "kwok_pod_rec12, 12 B per record in, 1 B status per record + 4 B handle per create back "
                "(kwok_ingest_pods_packed12)" if packed == 12 else
                "kwok_pod_rec, 20 B per record (kwok_ingest_pods_packed)" if packed else
                "kwok_pod_event, 48 B per record + dotted-quad strings (kwok_ingest_pods)",
        "link_bytes_per_step": (2 * n_churn * 12 + 2 * n_churn + 4 * n_churn if packed == 12 else
                                2 * n_churn * 20 + 2 * n_churn * 5 if packed else None),
        "value": trans / (ing + tck), "unit": "transitions/s (ingest + tick)",
        "ms_per_step": (ing + tck) / ticks * 1e3, "ingest_ms": ing / ticks * 1e3, "tick_ms": tck / ticks * 1e3,
        "median_ms": {"step": float(np.median([a + b for a, b in steps])) * 1e3,
                      "ingest": float(np.median([a for a, _ in steps])) * 1e3,
                      "tick": float(np.median([b for _, b in steps])) * 1e3},
        "steps_ms": [[round(a * 1e3, 3), round(b * 1e3, 3)] for a, b in steps],  # (ingest, tick) per step
        "ingest_records_per_s": recs * world / ing if ing else None,
        "tick_transitions_per_s": trans / tck if tck else None,
        "kernel_ms": kern / ticks, "emission_ms": emit / ticks,
        # multi-rank tick: the FRONT header to the (last) BACK launch's start -
        # allgather, and for long lists the host round trip, second allgather, k_pool_apply
        "exchange_ms": xch / ticks if (world > 1 or multi) else None,
        "phase_ms": phases,
        "roofline": c4_roofline(last, kern / ticks, once) if last else None,
        "counters_last_tick": last,
        "note": "ingest = kwok_ingest_pods: H2D of the records and their strings (page-locked batch buffers, "
                "kwok_host_alloc; batches over KWOK_INGEST_CHUNK records in chunks, each copied while the previous "
                "one is applied), the GPU event switch (prep, stable sort by bucket, per-bucket apply), D2H of the "
                "per-record handles / statuses / releases; event generation between steps untimed (the GPU idles "
                "~0.2 s there, so the first device work of a step can pay a clock ramp: medians beside means)"}


def c4_roofline(c, kern_ms, once=False):
    """the churn tick's kernels (k_tick + the job build + k_emit) against HBM: the
    steady tick's bytes (heartbeats - once: the node's state model only, one body
    - node and pod re-checks) + per Pending->Running patch POD_PATCH_BYTES + per
    deletion DELETE_BYTES, over the profiled tick's kernel time (HIP events
    around its launches).  once: traffic from the stored PMC passes of this
    kernel build (tools/gpu_c4once.sh), summed over the tick's kernels"""
    nb = NODE_STATE_BYTES if once else NODE_BYTES
    b = nb * c["heartbeat"] + POD_BYTES * c["pods_total"] + POD_PATCH_BYTES * c["pod_patch"] + DELETE_BYTES * c["delete"]
    ach = b / (kern_ms * 1e-3) / 1e9 if kern_ms else None
    out = {"bound": "hbm", "kernel": "k_tick + k_sparse_jobs + k_emit", "bytes_per_tick": b, "kernel_ms": kern_ms,
           "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS if ach else None,
           "byte_model": "per node %d B, per live pod %d B, per patch %d B, per delete %d B" % (
               nb, POD_BYTES, POD_PATCH_BYTES, DELETE_BYTES)}
    if once:
        tr, src = 0, []
        for k in ("k_tick", "k_sparse_jobs", "k_emit"):
            t, sname = stored_pmc(C4_PMC_FILE, k)
            if t is None:
                tr = None
                break
            tr += t
            src.append(sname)
        out["traffic"] = tr
        out["traffic_source"] = "; ".join(src) if tr else None
        out["traffic_ratio"] = tr / b if tr else None
    return out


def steady_queued(e, now, steps, warmup):
    """`steps` steady ticks queued two deep (kwok_tick_submit of tick k+1 before
    kwok_tick_collect of tick k) after `warmup` on the same path (the first
    queued submit allocates the second tick slot); returns (seconds, transitions,
    the clock after them)"""
    now += 30
    e.tick_submit(now)
    for w in range(max(warmup, 2)):
        if w + 1 < max(warmup, 2):
            now += 30
            e.tick_submit(now)
        e.tick_collect(read=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.tick_submit(now + 30)
    now += 30
    trans = 0
    for k in range(steps):
        if k + 1 < steps:
            e.tick_submit(now + 30)
            now += 30
        trans += transitions(e.tick_collect(read=False).counters)
    return time.perf_counter() - t0, trans, now


def stored_pmc(name, kernel):
    """HBM bytes per launch of `kernel` from a stored rocprofv3 FETCH_SIZE /
    WRITE_SIZE summary, if it was measured on THIS kernels.hip (else None)"""
    import hashlib
    pmc = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(pmc):
        return None, None
    d = json.load(open(pmc))
    ksha = hashlib.sha256(open(os.path.join(ROOT, "kwok_amd", "csrc", "kernels.hip"), "rb").read()).hexdigest()
    if d.get("kernels_sha256") != ksha:
        return None, None
    ks = [k for k in d["kernels"] if k == kernel or k.startswith("void %s<" % kernel) or k.startswith(kernel + "<")]
    if not ks:
        return None, None
    return d["kernels"][ks[0]]["hbm_bytes"], ("stored: profiles/%s, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per steady "
                                              "launch of %s on this kernel build (kernels.hip sha256 %s)"
                                              % (name, ks[0], ksha[:12]))


def heartbeat_once_leg(nodes, steps, warmup, churn_ticks, json_ticks=0):
    """The drop-in's engine: KWOK_CFG_HEARTBEAT_ONCE (engine_cgo.go), on the
    metric's fleet.  The tick materialises ONE heartbeat body (every node's
    patch is that body, node_controller.go:393-401) and the handle list, for
    callers that send one body to every node.  Legs: the initial tick (1M node
    inits + 10M Pending->Running patches), steady ticks queued (k_once: a
    heartbeat-once tick with nothing to emit, one wave per bucket), and C4
    churn ticks on the same engine."""
    e, fl, pods = workload.build_engine_fleet(keng.Engine, nodes, heartbeat_once=True)
    now = workload.S0 + 30
    e.profile_enable(True)
    t1 = time.perf_counter()
    r0 = e.tick(now, read=False)  # initial tick
    init_wall = time.perf_counter() - t1
    ph0, _ = e.profile_read()
    e.profile_enable(False)
    # the drop-in's read-back of that tick (ShimReader: lists + every patch byte, page-locked)
    t1 = time.perf_counter()
    init_read = ShimReader(e).read(r0)
    init_read_s = time.perf_counter() - t1
    dt, trans, now = steady_queued(e, now, steps, warmup)
    e.profile_enable(True)
    for _ in range(20):
        now += 30
        r = e.tick(now, read=False)
    ph, nt = e.profile_read()
    e.profile_enable(False)
    stats = e.stats()
    churn = cjson = None
    handoff = {}
    if churn_ticks:
        now, ch, churn = churn_leg(e, fl, pods, now, churn_ticks, nodes, once=True)
        now, ch, tog = churn_leg(e, fl, pods, now, churn_ticks, nodes, ch=ch, once=True, together=True)
        churn["together"] = {k: tog[k] for k in ("ms_per_step", "ingest_ms", "tick_ms", "median_ms", "kernel_ms",
                                                  "value", "unit")}
        churn["together"]["what"] = ("kwok_ingest_pods_packed12_tick: the tick queued behind the batch's apply "
                                     "passes (its kernels run while the results travel back), then kwok_tick_collect")
        for ov in (False, True):
            now, ch, handoff["overlapped" if ov else "sequential"] = churn_handoff_leg(e, fl, ch, now, max(3, churn_ticks),
                                                                                     nodes, ov)
        if json_ticks:
            now, _, cjson = churn_json_leg(e, fl, ch, now, json_ticks, nodes)
    e.close()
    lc = r.local_counters
    state_bytes = NODE_STATE_BYTES * lc[8] + POD_BYTES * lc[10]
    # what a k_once launch that reads the per-bucket summaries must move: a managed
    # node's state byte, one 16-byte summary per bucket, the heartbeat handle list
    # (4 B per managed node) and the one body
    once_bytes = NODE_SLOT_BYTES * lc[8] + 16 * workload.BUCKETS + 4 * r.counters[0] + 1072
    kern = ph["kernel"] / max(nt, 1)
    step_ms = dt / steps * 1e3
    # (the steady ticks' instance: k_once reading the per-bucket summaries, ONCE_SUM_USE = 2)
    traffic, traffic_src = stored_pmc(ONCE_PMC_FILE, "void k_once<false, 2u>")
    ilc = r0.local_counters
    init_bytes = INIT_BYTES * ilc[1] + POD_PATCH_BYTES * ilc[2]
    # the roofline over the queued step (kernel + the gap to the next launch), a lower
    # bound on the kernel's rate: a ~15 us kernel's HIP event pair reads a few us long;
    # the rocprofv3 kernel durations of this leg are committed under profiles/
    # (<round>_once_ktrace.txt, tools/gpu_full.sh)
    return {"workload": "metric configuration, KWOK_CFG_HEARTBEAT_ONCE (the cgo drop-in's engine: one heartbeat body "
                        "+ the handle list per tick); steady ticks queued", "steps": steps,
            "value": trans / dt, "unit": "transitions/s", "ms_per_step": step_ms,
            "kernel_ms_events": kern, "classify_ms": ph["classify"] / max(nt, 1),
            "tick_kernels": stats,
            "roofline": {"bound": "latency (two dependent round trips per bucket wave + the count atomics; "
                                  "launch-bound at this size)", "kernel": "k_once",
                         "bytes_per_launch": once_bytes,
                         "achieved": once_bytes / (step_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": once_bytes / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_per_step_gbs": traffic / (step_ms * 1e-3) / 1e9 if traffic else None,
                         "timing": "queued step time (launch-to-launch), not the event pair",
                         "note": "bytes: what a launch reading the per-bucket summaries moves (node state bytes, "
                                 "16 B per bucket, 4 B per heartbeat handle, one body; DESIGN.md §16). The state "
                                 "model of SURVEY 8(d) (node 9 + 9 B, pod 10 B per tick) is state_model_bytes: the "
                                 "summaries make reading it unnecessary while no pod state changes",
                         "state_model_bytes": state_bytes,
                         "state_model_equiv_gbs": state_bytes / (step_ms * 1e-3) / 1e9},
            "initial_tick": {"wall_ms": init_wall * 1e3, "kernel_ms": ph0["kernel"], "emission_ms": ph0["emit_kernel"],
                             "transitions": transitions(r0.counters),
                             "with_handoff": {"ms": (init_wall + init_read_s) * 1e3, "read_ms": init_read_s * 1e3,
                                              "bytes_to_host": init_read[0], "pieces": init_read[1],
                                              "link_gbs": init_read[0] / init_read_s / 1e9,
                                              "what": "the tick, then the drop-in's read-back (ShimReader: lists, one "
                                                      "heartbeat body, every node-init and pod patch byte in 64 MiB "
                                                      "pieces into page-locked memory)"},
                             "emit_roofline": {"kernel": "k_pod_jobs + k_emit", "bytes": init_bytes,
                                               "achieved": init_bytes / (ph0["emit_kernel"] * 1e-3) / 1e9
                                               if ph0["emit_kernel"] else None,
                                               "frac": init_bytes / (ph0["emit_kernel"] * 1e-3) / 1e9 / HBM_PEAK_GBS
                                               if ph0["emit_kernel"] else None}},
            "churn": None if churn is None else dict({k: churn[k] for k in (
                "workload", "ms_per_step", "ingest_ms", "tick_ms", "median_ms", "kernel_ms", "emission_ms", "value",
                "unit", "tick_transitions_per_s", "roofline", "phase_ms", "together")}, with_handoff=handoff),
            "churn_json": cjson}


def churn_json_leg(e, fl, ch, now, ticks, n_churn):
    """C4 from the documents themselves: per tick the 2 x n_churn pod documents
    a watch carries (workload.ChurnJson: the deletion-marked Running pods as
    kwok patched them, ~1.6 KB, and the scheduled Pending creates, ~1.1 KB),
    decoded on the GPU and routed there (kwok_ingest_pods_json), then the tick.
    Beside it: the host codec (kwok_decode_pods, all host threads) on one such
    batch - the drop-in's other path from the same documents."""
    from kwok_amd.codec import Codec
    codec = Codec(manage_all_nodes=True)
    ch = workload.ChurnJson.from_churn(ch, workload.node_names_by_handle(fl), alloc=keng.host_array)  # (its live pods)
    dump = lambda: e.dump_pods(0, workload.BUCKETS * fl.cp)  # noqa: E731
    outs = (keng.host_array((2 * n_churn,), np.int32), keng.host_array((2 * n_churn,), np.int32),
            keng.host_array((2 * n_churn,), np.uint32))
    steps, host = [], None
    trans = n_host = docs = nbytes = 0
    rd = ShimReader(e)
    reads = []
    for k in range(ticks + 1):
        arena, offs, lens, ops, handles = ch.batch_json(dump, now)
        if k == 0:  # the host codec on this batch (untimed leg warmup)
            t0 = time.perf_counter()
            h = workload.host_decode_arrays(codec, arena, offs, lens, threads=os.cpu_count() and min(16, os.cpu_count()))
            host = (time.perf_counter() - t0, int((h["status"] == 0).sum()))
            del h
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hs, st, _rel, nh = e.ingest_pods_json(codec, arena, offs, lens, ops, handles, out=outs)
        t1 = time.perf_counter()
        r = e.tick(now, read=False)
        t2 = time.perf_counter()
        t3 = time.perf_counter()
        rd.read(r)  # the drop-in's read-back: every list and patch byte (ShimReader)
        t4 = time.perf_counter()
        ch.applied(hs.copy(), st)
        now += 30
        if k:
            reads.append(t4 - t3)
            steps.append((t1 - t0, t2 - t1))
            trans += transitions(r.counters)
            n_host += nh
            docs += len(offs)
            nbytes += int(lens.sum())
    ing = sum(a for a, _ in steps)
    tck = sum(b for _, b in steps)
    codec.close()
    return now, ch, {
        "workload": "C4 from JSON: %d deletion-marked + %d created pod documents per tick on the metric fleet "
                    "(heartbeat-once engine)" % (n_churn, n_churn),
        "ticks": ticks, "documents_per_tick": docs // max(ticks, 1), "json_bytes_per_tick": nbytes // max(ticks, 1),
        "value": trans / (ing + tck), "unit": "transitions/s (decode + ingest + tick)",
        "ms_per_step": (ing + tck) / ticks * 1e3, "decode_ingest_ms": ing / ticks * 1e3, "tick_ms": tck / ticks * 1e3,
        "median_ms": {"step": float(np.median([a + b for a, b in steps])) * 1e3,
                      "decode_ingest": float(np.median([a for a, _ in steps])) * 1e3},
        "documents_per_s": docs / ing if ing else None, "documents_decided_by_host": n_host,
        "with_handoff_ms": (ing + tck + sum(reads)) / ticks * 1e3, "read_back_ms": sum(reads) / ticks * 1e3,
        "host_codec": {"ms": host[0] * 1e3, "documents_per_s": len(offs) / host[0], "threads": min(16, os.cpu_count()),
                       "what": "kwok_decode_pods (codec.cpp) on one batch of the same documents, records only "
                               "(no ingest): the drop-in's host path"},
        "note": "decode_ingest = kwok_ingest_pods_json: the documents (page-locked) copied to HBM, k_json_pods (one "
                "thread per document), then kwok_ingest_pods' GPU event switch over the decoded records"}


def c2_leg(steps, warmup):
    """BASELINE configs[1] at its own size (100k nodes x 1M pods, one MI355X):
    steady ticks queued, full heartbeat bodies and heartbeat-once"""
    out = {}
    for once in (False, True):
        e, fl, _ = workload.build_engine_fleet(keng.Engine, 100_000, heartbeat_once=once)
        now = workload.S0 + 30
        e.tick(now, read=False)
        dt, trans, now = steady_queued(e, now, steps, warmup)
        out["heartbeat_once" if once else "full_bodies"] = {"value": trans / dt, "ms_per_step": dt / steps * 1e3,
                                                            "tick_kernels": e.stats()}
        e.close()
    out["workload"] = "BASELINE configs[1]: 100k nodes x 1M pods steady heartbeat + status ticks, 1x MI355X, queued"
    out["unit"] = "transitions/s"
    return out


def emulated_ranks_leg(nodes, ranks, steps, churn_ticks):
    """The per-rank cost of the multi-rank exchange at N = `ranks`, on one GPU:
    a one-rank engine on the FRONT / RCCL allgather / BACK path
    (KWOK_FORCE_MULTI) whose BACK launch folds `ranks` exchange messages - its
    own and `ranks` - 1 copies with their addresses moved inside the CIDR
    (KWOK_EMULATE_RANKS) - so every tick commits `ranks` ranks' Gets and applies
    their Uses and Puts to the replicated pool, as each rank of an N-GPU run
    does.  The fleet is one rank's (1M x 10M) under the CIDR an
    N-rank fleet takes.  Steady ticks (queued) and C4 churn ticks (1M + 1M per
    rank per tick: `ranks` x 1M releases and Gets per tick at every rank).
    Diagnostics: the pool's addresses stop matching a real fleet after the
    first emulated tick, so nothing here is checked against the oracle."""
    env = {"KWOK_FORCE_MULTI": "1", "KWOK_EMULATE_RANKS": str(ranks)}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e, fl, pods = workload.build_engine_fleet(keng.Engine, nodes, comm_id=keng.comm_id(),
                                                  cidr=cidr_for(nodes * workload.PODS_PER_NODE * ranks))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    now = workload.S0 + 30
    e.tick(now, read=False)
    for _ in range(3):
        now += 30
        e.tick(now, read=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        now += 30
        e.tick(now, read=False)
    dt = (time.perf_counter() - t0) / steps
    # the same steady ticks queued two deep, as the headline's (kwok_tick_submit of tick
    # k+1 before kwok_tick_collect of tick k: no host round trip between ticks)
    dq, _, now = steady_queued(e, now, steps, 3)
    e.profile_enable(True)
    for _ in range(10):
        now += 30
        e.tick(now, read=False)
    ph, nt = e.profile_read()
    e.profile_enable(False)
    churn = None
    if churn_ticks:
        now, _, churn = churn_leg(e, fl, pods, now, churn_ticks, nodes, multi=True)  # (a one-rank multi engine)
    e.close()
    return {"ranks": ranks, "workload": "one rank's 1M x 10M fleet; BACK folds %d ranks' exchange messages and lists "
                                        "(KWOK_FORCE_MULTI + KWOK_EMULATE_RANKS, one-rank RCCL allgather)" % ranks,
            "steady_ms_per_tick": dt * 1e3, "steady_queued_ms_per_tick": dq / steps * 1e3,
            "steady_phase_ms": {k: v / max(nt, 1) for k, v in ph.items()},
            "churn": None if churn is None else {k: churn[k] for k in ("ms_per_step", "ingest_ms", "tick_ms",
                                                                       "kernel_ms", "exchange_ms", "median_ms",
                                                                       "phase_ms")},
            "note": "steady_ms_per_tick: blocking kwok_tick steps; steady_queued_ms_per_tick: the headline's "
                    "queued steps; the allgather is a one-rank copy (the xGMI transfer of N ranks' 8 KiB messages / "
                    "MB lists is not in it)"}


def flap_leg(nodes, ticks, heartbeat_once=False):
    """BASELINE configs[4] (C5): a fleet of `nodes` nodes x 10 pods with
    ManageAllNodes=false (annotation selector on 50% of the nodes, disregard
    annotation on 0.1%); per tick 1% of the managed nodes are deleted and
    created again (workload.Flap).  A step = kwok_ingest_nodes of that batch +
    one kwok_tick (heartbeats of the managed half, the flapped nodes' init
    patches, re-evaluation of the managed nodes' pods).  First step warmup."""
    e, fl, _ = workload.build_engine_fleet(keng.Engine, nodes, managed_frac=0.5, lockable_frac=0.999, seed=5,
                                           heartbeat_once=heartbeat_once)
    now = workload.S0 + 30
    e.tick(now, read=False)
    f = workload.Flap(fl, 0.01, seed=6)
    ing = tck = 0.0
    trans = 0
    last = None
    outs = (keng.host_array((2 * f.k,), np.int32), keng.host_array((2 * f.k,), np.int32))
    for k in range(ticks + 1):
        now += 30
        # the batch as a watch client holds it: its own arena of the names, page-locked
        ev, ar = f.batch(compact=True, alloc=keng.host_array)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.ingest_nodes_raw(ev, ar, out=outs)
        t1 = time.perf_counter()
        r = e.tick(now, read=False)
        t2 = time.perf_counter()
        if k:
            ing += t1 - t0
            tck += t2 - t1
            trans += transitions(r.counters)
            last = dict(zip(abi.COUNTERS, list(r.counters)))
    js = flap_json(e, f, now, ticks) if heartbeat_once else None
    e.close()
    return {"workload": "C5 node flap under partial management (BASELINE configs[4]): %d nodes x %d pods, "
                        "annotation selector on 50%%, 1%% of the managed nodes deleted + re-added per tick%s"
                        % (nodes, nodes * workload.PODS_PER_NODE, ", KWOK_CFG_HEARTBEAT_ONCE" if heartbeat_once else ""),
            "ticks": ticks, "flapped_nodes_per_tick": f.k,
            "value": trans / (ing + tck), "unit": "transitions/s (ingest + tick)",
            "ms_per_step": (ing + tck) / ticks * 1e3, "ingest_ms": ing / ticks * 1e3, "tick_ms": tck / ticks * 1e3,
            "counters_last_tick": last, "from_json": js}


def flap_json(e, f, now, ticks):
    """C5 from the node documents a watch carries (kwok_ingest_nodes_json: decoded on
    the GPU, Deleted events' statuses not read, Added nodes with a zero status), then
    the tick; the same flap generator continued on the same engine"""
    from kwok_amd.codec import Codec
    codec = Codec(manage_all_nodes=False, manage_nodes_with_annotation_selector="kwok.x-k8s.io/node=fake",
                  disregard_status_with_annotation_selector="kwok.x-k8s.io/status=custom")
    ing = tck = 0.0
    n_host = docs = nbytes = 0
    for k in range(ticks + 1):
        now += 30
        arena, offs, lens, ops, _ = f.batch_json()
        ap = keng.host_array((len(arena),), np.uint8)  # (page-locked, as the Go shim stages the documents)
        ap[:] = np.frombuffer(arena, np.uint8)
        arena = ap
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hs, st, nh = e.ingest_nodes_json(codec, arena, offs, lens, ops)
        t1 = time.perf_counter()
        e.tick(now, read=False)
        t2 = time.perf_counter()
        if k:
            ing += t1 - t0
            tck += t2 - t1
            n_host += nh
            docs += len(offs)
            nbytes += int(lens.sum())
    codec.close()
    return {"ms_per_step": (ing + tck) / ticks * 1e3, "decode_ingest_ms": ing / ticks * 1e3, "tick_ms": tck / ticks * 1e3,
            "documents_per_tick": docs // ticks, "json_bytes_per_tick": nbytes // ticks,
            "documents_decided_by_host": n_host,
            "note": "kwok_ingest_nodes_json: the documents (page-locked) copied to HBM, k_json_nodes (one thread per "
                    "document), kwok_ingest_nodes' GPU event switch over the records"}


class ShimReader:
    """What the Go drop-in reads back after a tick (engine_cgo.go tick /
    applyPatches): the lists (kwok_read_outputs without an
    arena: heartbeat handles only when their epoch changed, node-init / pod-patch
    handles with offsets and lengths, the delete list), ONE heartbeat body, then
    every node-init and pod patch byte in pieces of at most READ_CHUNK bytes
    (kwok_read_arena), all into page-locked host memory (kwok_host_alloc).  The
    apply callback gets views of the staging buffer (no copy here; the Go shim
    hands them to its PATCH pool).  asynchronous=True: the pieces are queued with
    kwok_read_arena_async into one staging buffer of the tick's patch bytes and
    waited for later (read_wait), so the next batch's ingest and tick run under
    the device-to-host copy."""

    READ_CHUNK = 64 << 20  # engine_cgo.go readChunk

    def __init__(self, e, asynchronous=False):
        self.e = e
        self.asynchronous = asynchronous
        self.epoch = None
        self.bufs = {}

    def buf(self, name, n, dt):
        b = self.bufs.get(name)
        if b is None or b.size < n:
            b = self.bufs[name] = keng.host_array((max(int(n * 1.25), 1),), dt)
        return b

    def read(self, res):
        """returns (bytes over the link, arena pieces)"""
        e = self.e
        hb = self.buf("hb", res.n_heartbeat, np.int32) if res.heartbeat_epoch != self.epoch else None
        self.epoch = res.heartbeat_epoch
        ini, ini_off, ini_len = (self.buf("ini", res.n_node_init, np.int32), self.buf("ini_off", res.n_node_init, np.uint64),
                                 self.buf("ini_len", res.n_node_init, np.uint32))
        pp, pp_off, pp_len = (self.buf("pp", res.n_pod_patch, np.int32), self.buf("pp_off", res.n_pod_patch, np.uint64),
                              self.buf("pp_len", res.n_pod_patch, np.uint32))
        dl, dlf = self.buf("dl", res.n_delete, np.int32), self.buf("dlf", res.n_delete, np.uint8)
        out = abi.Outputs(hb.ctypes.data if hb is not None else None, 0, ini.ctypes.data, ini_off.ctypes.data,
                          ini_len.ctypes.data, pp.ctypes.data, pp_off.ctypes.data, pp_len.ctypes.data,
                          dl.ctypes.data, dlf.ctypes.data, None, 0, 0)
        e._check(e._lib.kwok_read_outputs(e._h, C.byref(out)), "read_outputs (lists)")
        nbytes = (res.n_heartbeat * 4 if hb is not None else 0) + res.n_node_init * 16 + res.n_pod_patch * 16 + \
            res.n_delete * 5
        pieces = 0
        if res.n_heartbeat:
            body = self.buf("body", res.heartbeat_len, np.uint8)
            e.read_arena(out.heartbeat_off, res.heartbeat_len, body)
            nbytes += res.heartbeat_len
        total = sum(int(ln[:n].sum()) for n, ln in ((res.n_node_init, ini_len), (res.n_pod_patch, pp_len)))
        stage = self.buf("stage", total if self.asynchronous else self.READ_CHUNK, np.uint8)
        at = 0
        for n, offs, lens in ((res.n_node_init, ini_off, ini_len), (res.n_pod_patch, pp_off, pp_len)):
            if not n:
                continue
            offs, ends = offs[:n], offs[:n].astype(np.int64) + lens[:n]
            i = 0
            while i < n:  # the shim's greedy pieces: consecutive patches within READ_CHUNK bytes
                lo = int(offs[i])
                j = max(i + 1, int(np.searchsorted(ends, lo + self.READ_CHUNK, side="right")))
                ln = int(ends[j - 1]) - lo
                if self.asynchronous:
                    e.read_arena_async(lo, ln, stage[at:at + ln])
                    at += ln
                else:
                    e.read_arena(lo, ln, stage)
                nbytes += ln
                pieces += 1
                i = j
        return nbytes, pieces

    def wait(self):
        self.e.read_wait()


def churn_handoff_leg(e, fl, ch, now, ticks, n_churn, overlap):
    """C4 as the drop-in runs it (heartbeat-once engine): ingest + tick + the
    shim's read-back of every list and patch byte (ShimReader).  overlap=False:
    one after the other.  overlap=True: tick k's pieces are queued
    (kwok_read_arena_async) at the start of step k+1 and waited for at its end, so
    the device-to-host copy runs beside batch k+1's ingest (host-to-device) and
    tick; the step is then bounded by the larger of the two.  Batch generation
    (which reads the pod states back) sits between the timed steps."""
    outs = (keng.host_array((n_churn,), np.int32), keng.host_array((2 * n_churn,), np.int8), None)
    rd = ShimReader(e, asynchronous=overlap)
    dump = lambda: e.dump_pods(0, workload.BUCKETS * fl.cp)  # noqa: E731
    ch.packed, ch.bufs = 12, None
    steps, nbytes, pieces, trans = [], 0, 0, 0
    pending = None
    warm = 2 if overlap else 1  # (overlapped: step 1 reads tick 0 into freshly pinned staging)
    for k in range(ticks + warm):
        ev, _ = ch.batch(dump, now)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if pending is not None:  # tick k-1's read, queued beside this step's work
            nb, pc = rd.read(pending)
        hs, st, _ = e.ingest_pods_packed12(ev, new_cap=len(ev) // 2, out=outs)
        r = e.tick(now, read=False)
        if overlap:
            if pending is not None:
                rd.wait()
            pending = r
        else:
            nb, pc = rd.read(r)
        dt = time.perf_counter() - t0
        ch.applied(hs.copy(), st, new_only=True)
        now += 30
        if k >= warm:  # (step 0: warmup; overlapped, it also has no earlier tick to read)
            steps.append(dt)
            nbytes += nb
            pieces += pc
            trans += transitions(r.counters)
    if overlap:  # (the last tick's read: done outside the timed steps)
        rd.read(pending)
        rd.wait()
    ms = float(np.mean(steps)) * 1e3
    return now, ch, {"overlap": overlap, "ticks": len(steps), "ms_per_step": ms,
                     "median_ms": float(np.median(steps)) * 1e3,
                     "bytes_to_host_per_step": nbytes / len(steps), "pieces_per_step": pieces / len(steps),
                     "link_gbs_equivalent": nbytes / len(steps) / (ms * 1e-3) / 1e9,
                     "value": trans / sum(steps), "unit": "transitions/s (ingest + tick + read-back)"}


class Handoff:
    """The per-tick hand-off a Go caller consumes: compact
    arena (one heartbeat body + the patch region), patch / delete lists, and the
    heartbeat handle list only when its epoch changed."""

    def __init__(self, e):
        self.e = e
        self.epoch = None
        self.bufs = {}

    def buf(self, name, n, dt):
        b = self.bufs.get(name)
        if b is None or b.size < n:
            b = self.bufs[name] = np.empty(max(n, 1), dt)
        return b

    def read(self, res):
        hb = self.buf("hb", res.n_heartbeat, np.int32) if res.heartbeat_epoch != self.epoch else None
        self.epoch = res.heartbeat_epoch
        arena = self.buf("arena", res.arena_bytes - (res.n_heartbeat - 1) * res.heartbeat_stride
                         if res.n_heartbeat else res.arena_bytes, np.uint8)
        p = lambda name, n, dt: self.buf(name, n, dt).ctypes.data  # noqa: E731
        out = abi.Outputs(hb.ctypes.data if hb is not None else None, 0,
                          p("ini", res.n_node_init, np.int32), p("ini_off", res.n_node_init, np.uint64),
                          p("ini_len", res.n_node_init, np.uint32),
                          p("pp", res.n_pod_patch, np.int32), p("pp_off", res.n_pod_patch, np.uint64),
                          p("pp_len", res.n_pod_patch, np.uint32),
                          p("dl", res.n_delete, np.int32), p("dlf", res.n_delete, np.uint8),
                          arena.ctypes.data, arena.nbytes, abi.READ_HEARTBEAT_ONCE)
        self.e._check(self.e._lib.kwok_read_outputs(self.e._h, C.byref(out)), "read_outputs")
        return out.arena_copied


def main():
    a = parse()
    # stdout carries exactly one JSON line: libraries that print banners to the C
    # stdout (RCCL prints "RCCL version ..." at communicator init) go to stderr
    sys.stdout.flush()
    json_out = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if a.leg:  # a child process of leg(): one secondary leg, its JSON on stdout
        torch.cuda.set_device(0)
        os.write(json_out, (json.dumps(run_leg(a.leg, a)) + "\n").encode())
        return
    local = 0 if REHEARSAL else int(os.environ.get("LOCAL_RANK", "0"))
    if REHEARSAL:
        os.environ.setdefault("KWOK_TICK_BLOCKS_PER_CU", "1")
    if world > 1:
        dist.init_process_group("gloo")  # control plane only; the data path uses the engine's RCCL comm

    comm = None
    gather = None
    if world > 1 and REHEARSAL:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from dist_common import gloo_allgather_fn  # rehearsal only: host-memory exchange
        gather = gloo_allgather_fn()
    elif world > 1:
        obj = [keng.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = obj[0]
    elif os.environ.get("KWOK_FORCE_MULTI"):  # diagnostics: one rank through FRONT / RCCL exchange / BACK
        comm = keng.comm_id()
    total_pods = a.nodes_per_rank * world * workload.PODS_PER_NODE
    cidr = cidr_for(total_pods)
    t0 = time.perf_counter()
    e, fl, pods = workload.build_engine_fleet(keng.Engine, a.nodes_per_rank, rank=rank, world=world, device=local,
                                              comm_id=comm, allgather=gather, cidr=cidr)
    setup_s = time.perf_counter() - t0

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    # ---- initial tick (untimed warmup step 0, measured on its own) ----------
    now = workload.S0 + 30
    barrier()
    e.profile_enable(True)
    e.profile_host(reset=True)
    t1 = time.perf_counter()
    r0 = e.tick(now, read=False)
    init_wall = max_over_ranks(time.perf_counter() - t1)
    init_host, _ = e.profile_host(reset=True)
    ph0, _ = e.profile_read()
    e.profile_enable(False)
    first = dict(zip(abi.COUNTERS, list(r0.counters)))
    now += 30
    # the remaining warmup steps take the timed steps' path (queued two deep), so
    # the second tick slot (its lists and ~8 GB arena) is allocated before timing
    if a.warmup > 1:
        e.tick_submit(now)
        now += 30
        for w in range(1, a.warmup):
            if w + 1 < a.warmup:
                e.tick_submit(now)
                now += 30
            e.tick_collect(read=False)

    # ---- timed steps: queued submit / collect ----------------------------------
    barrier()
    e.profile_host(reset=True)
    t0 = time.perf_counter()
    trans = evald = 0
    last = None
    e.tick_submit(now)
    now += 30
    for k in range(a.steps):
        if k + 1 < a.steps:
            e.tick_submit(now)
            now += 30
        r = e.tick_collect(read=False)
        c = r.counters
        trans += transitions(c)
        evald += c[6] + c[7]
        last = r
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    host_ms, host_n = e.profile_host(reset=True)

    # ---- the same steps, one blocking kwok_tick each ---------------------------
    barrier()
    t1 = time.perf_counter()
    for k in range(a.steps):
        e.tick(now, read=False)
        now += 30
    barrier()
    dt_sync = max_over_ranks(time.perf_counter() - t1)

    # ---- the same steps with the per-tick hand-off (queued) --------------------
    ho = Handoff(e)
    copied = trans_read = 0
    barrier()
    t1 = time.perf_counter()
    e.tick_submit(now)
    now += 30
    for k in range(a.steps):
        if k + 1 < a.steps:
            e.tick_submit(now)
            now += 30
        r = e.tick_collect(read=False)
        trans_read += transitions(r.counters)
        copied += ho.read(r)
    barrier()
    dt_read = max_over_ranks(time.perf_counter() - t1)

    # ---- roofline pass: HIP events around each k_tick launch ------------------
    e.profile_enable(True)
    for k in range(a.roofline_ticks):
        e.tick(now, read=False)
        now += 30
    phases, nt = e.profile_read()
    e.profile_enable(False)

    churn = churn_ev = None
    if a.churn_ticks > 0:
        now, ch, churn = churn_leg(e, fl, pods, now, a.churn_ticks, a.churn or a.nodes_per_rank, rank, world,
                                   barrier, max_over_ranks, multi=comm is not None or gather is not None)
        if world == 1 and comm is None and gather is None:  # the batch with its tick behind it (one call)
            now, ch, tog = churn_leg(e, fl, pods, now, a.churn_ticks, a.churn or a.nodes_per_rank, ch=ch,
                                     together=True)
            churn["together"] = {k: tog[k] for k in ("ms_per_step", "ingest_ms", "tick_ms", "median_ms", "kernel_ms",
                                                      "value", "unit")}
            churn["together"]["what"] = ("kwok_ingest_pods_packed12_tick: the tick queued behind the batch's apply "
                                         "passes, then kwok_tick_collect")
        if world == 1:  # the same storm through the full record form, beside it
            now, ch, churn_ev = churn_leg(e, fl, pods, now, max(2, a.churn_ticks // 2), a.churn or a.nodes_per_rank,
                                          rank, world, barrier, max_over_ranks, packed=False, ch=ch)

    e.close()
    flap = leg("flap", a) if world == 1 and a.flap_ticks > 0 else None
    flap_once = leg("flap_once", a) if world == 1 and a.flap_ticks > 0 and a.once_ticks else None
    hb_once = leg("hb_once", a) if world == 1 and a.once_ticks else None
    c2 = leg("c2", a) if world == 1 and a.c2 and a.nodes_per_rank == NODES_PER_RANK else None
    emul = leg("emul", a) if world == 1 and a.emulate_ranks > 1 and not REHEARSAL else None

    if rank == 0:
        kern_ms = phases["kernel"] / max(nt, 1)
        classify_ms = phases["classify"] / max(nt, 1)
        lc = last.local_counters
        n_nodes, n_pods = lc[8], lc[10]  # nodes_managed, pods_total (this rank)
        alg_bytes = NODE_BYTES * n_nodes + POD_BYTES * n_pods
        state_bytes = NODE_STATE_BYTES * n_nodes + POD_BYTES * n_pods
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
        traffic, traffic_src = stored_pmc(PMC_FILE, "k_tick") if a.nodes_per_rank == NODES_PER_RANK else (None, None)
        ilc = r0.local_counters
        init_bytes = INIT_BYTES * ilc[1] + POD_PATCH_BYTES * ilc[2]
        emit_ms = ph0["emit_kernel"]
        out = {
            "metric": "state transitions/sec at 1M nodes/10M pods, 1-8 MI355X; % HBM roofline",
            "value": trans / dt,
            "unit": "transitions/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "metric configuration: 1M nodes x 10M pods per GPU, steady-state heartbeat + "
                                   "status ticks (configs[1]'s tick at the metric's size)",
                       "nodes": fl.total_nodes, "pods": fl.total_nodes * workload.PODS_PER_NODE,
                       "nodes_per_gpu": a.nodes_per_rank, "pods_per_node": workload.PODS_PER_NODE,
                       "cidr": cidr, "buckets": workload.BUCKETS, "parallelism": "bucket-sharded x%d" % world},
            "tick_api": "kwok_tick_submit/kwok_tick_collect, tick k+1 queued before tick k is collected",
            "ms_per_step_kwok_tick": dt_sync / a.steps * 1e3,
            "ms_per_step_with_handoff": dt_read / a.steps * 1e3,
            "handoff": {"transitions_per_s": trans_read / dt_read,
                        "bytes_to_host_per_step": copied / a.steps,
                        "what": "kwok_read_outputs with KWOK_READ_HEARTBEAT_ONCE (one heartbeat body + patch "
                                "region + lists; heartbeat handles only when the epoch changes), pageable host "
                                "buffers, queued ticks"},
            "objects_evaluated_per_s": evald / dt,
            "phase_ms_per_tick": {k: v / max(nt, 1) for k, v in phases.items()},
            "host_ms_per_tick": {k: v / max(host_n, 1) for k, v in host_ms.items()},
            "initial_tick": {"wall_ms": init_wall * 1e3, "kernel_ms": ph0["kernel"], "emission_ms": emit_ms,
                             "host_ms": init_host,
                             "transitions": transitions(r0.counters),
                             "transitions_per_s": transitions(r0.counters) / init_wall,
                             "counters": first,
                             "emit_roofline": {"bound": "hbm", "kernel": "k_pod_jobs + k_emit (the emission pipeline)",
                                               "bytes": init_bytes,
                                               "achieved": init_bytes / (emit_ms * 1e-3) / 1e9 if emit_ms else None,
                                               "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                               "frac": init_bytes / (emit_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                               if emit_ms else None}},
            "setup_s": setup_s,
            "roofline": {"bound": "hbm", "kernel": "k_tick", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_launch": alg_bytes, "avg_launch_ms": kern_ms, "traffic_source": traffic_src,
                         "timing": "HIP events around each k_tick launch (hipExtLaunchKernelGGL), %d ticks" % nt},
            "state_only": {"bytes_per_tick": state_bytes,
                           "achieved": state_bytes / (classify_ms * 1e-3) / 1e9 if classify_ms > 0 else 0.0,
                           "unit": "GB/s", "classify_ms": classify_ms,
                           "note": "SoA state read + written per tick without the materialised heartbeat bodies, "
                                   "over the classification phase (first chain block start to the last arrival, "
                                   "kernel clock stamps), which runs under the heartbeat stream"},
        }
        if REHEARSAL:
            out["rehearsal"] = "all ranks on GPU 0, host allgather instead of RCCL: not a reported measurement"
        if churn is not None:
            out["churn"] = churn
        if churn_ev is not None:
            out["churn_events"] = churn_ev
        if flap is not None:
            out["flap"] = flap
        if hb_once is not None:
            if flap_once is not None:
                hb_once["flap"] = flap_once
            out["heartbeat_once"] = hb_once
        if c2 is not None:
            out["c2"] = c2
        if emul is not None:
            out["emulated_ranks"] = emul
        if world == 1 and a.cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.nodes_per_rank, a.cpu_threads, a.cpu_ticks)
        sys.stdout.flush()
        os.write(json_out, (json.dumps(out) + "\n").encode())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
