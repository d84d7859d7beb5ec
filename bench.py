#!/usr/bin/env python3
"""bench.py - kwok fake-kubelet tick on MI355X (BASELINE.json metric:
state transitions/sec, % of HBM roofline).

Workload (N=1): configs[1] of BASELINE.json - 100k nodes x 1M pods, steady-state
heartbeat + status ticks on one MI355X.  Weak scaling: every rank owns 100k
nodes / 1M pods of a fleet of N x 100k nodes hashed into 4096 buckets
(contiguous bucket ranges per rank), and ranks exchange pool/counter data over
RCCL each tick.  A step = one tick (one heartbeat interval at a fixed clock):
heartbeat patches for every managed node, lock checks for every node,
re-evaluation of every pod, ipPool bookkeeping, and the host collecting the
tick's result.  Steps are queued (kwok_tick_submit for tick k+1 before
kwok_tick_collect of tick k, outputs double-buffered); --no-queue times one
blocking kwok_tick per step, and that figure is always reported beside the
queued one (ms_per_step_kwok_tick).  Warmup includes the initial tick (100k
node-init patches + 1M Pending->Running patches with IP allocation).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
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
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))

from kwok_amd import engine as keng  # noqa: E402
from kwok_amd import workload  # noqa: E402

keng.load_engine_lib()

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
NODES_PER_RANK = 100_000
# algorithmic HBM bytes of one tick (SURVEY.md §8(d) byte model):
# per managed node a heartbeat (1 B flags + 4 B hb-time + 4 B out-index + the
# 1059-byte materialised patch = 1068 B) and a no-op re-lock check (9 B); per
# live pod a no-op re-check (10 B)
HB_BYTES = 1059
NODE_BYTES = 1068 + 9
POD_BYTES = 10
PMC_FILE = "r1e_pmc_tick.json"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nodes-per-rank", type=int, default=NODES_PER_RANK)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 (N=1)")
    ap.add_argument("--cpu-nodes", type=int, default=NODES_PER_RANK)
    ap.add_argument("--roofline-ticks", type=int, default=20)
    ap.add_argument("--no-queue", dest="queue", action="store_false",
                    help="time kwok_tick one at a time instead of queued submit/collect")
    return ap.parse_args()


def cpu_baseline(nodes, ticks=5):
    """The C oracle (a sequential restatement of the reference controllers)
    on one host core, same workload shape, bounded to a few steady ticks."""
    from oracle.oracle import Oracle  # test infrastructure: baseline only
    t0 = time.perf_counter()
    o, _, _ = workload.build_engine_fleet(Oracle, nodes)
    o.tick(workload.S0 + 30, read=False)  # initial tick (locks + Pending->Running)
    t_init = time.perf_counter() - t0
    t1 = time.perf_counter()
    trans = 0
    for k in range(ticks):
        r = o.tick(workload.S0 + 60 + 30 * k, read=False)
        trans += r.counters[0] + r.counters[1] + r.counters[2] + r.counters[3] + r.counters[5]
    dt = time.perf_counter() - t1
    o.close()
    return {"value": trans / dt, "unit": "transitions/s", "cores": 1, "kind": "port",
            "sample": "oracle (C restatement), %d nodes x %d pods, %d steady ticks after the initial tick "
                      "(setup+initial tick %.1fs)" % (nodes, nodes * 10, ticks, t_init),
            "ms_per_step": dt / ticks * 1e3}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")  # control plane only; the data path uses the engine's RCCL comm

    comm = None
    if world > 1:
        obj = [keng.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = obj[0]
    t0 = time.perf_counter()
    e, fl, pods = workload.build_engine_fleet(keng.Engine, a.nodes_per_rank, rank=rank, world=world, device=local,
                                              comm_id=comm)
    setup_s = time.perf_counter() - t0

    now = workload.S0 + 30
    first = None
    for w in range(a.warmup):
        r = e.tick(now, read=False)
        if w == 0:
            first = dict(zip(keng.abi.COUNTERS, list(r.counters)))
        now += 30

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e.profile_host(reset=True)
    t0 = time.perf_counter()
    trans = evald = 0
    last = None
    if a.queue:
        # tick k+1 is submitted before tick k is collected (kwok_tick_submit /
        # kwok_tick_collect): the next launch is queued while the host finishes a tick
        e.tick_submit(now)
        now += 30
    for k in range(a.steps):
        if not a.queue:
            r = e.tick(now, read=False)
            now += 30
        else:
            if k + 1 < a.steps:
                e.tick_submit(now)
                now += 30
            r = e.tick_collect(read=False)
        c = r.counters
        trans += c[0] + c[1] + c[2] + c[3] + c[5]
        evald += c[6] + c[7]
        last = r
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    host_ms, host_n = e.profile_host(reset=True)
    # the same steps one kwok_tick at a time (reported beside the queued figure)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for k in range(a.steps):
        e.tick(now, read=False)
        now += 30
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt_sync = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([dt_sync], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_sync = float(t[0])
    # roofline pass: the same ticks with HIP events around each k_tick launch
    # (kernel-exact hipExtLaunchKernelGGL events) and the kernel's phase stamps
    e.profile_enable(True)
    for k in range(a.roofline_ticks):
        e.tick(now, read=False)
        now += 30
    phases, nt = e.profile_read()
    e.profile_enable(False)

    if rank == 0:
        kern_ms = phases["kernel"] / max(nt, 1)
        lc = last.local_counters
        alg_bytes = NODE_BYTES * lc[8] + POD_BYTES * lc[10]  # nodes_managed, pods_total (this rank)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
        traffic, traffic_src = None, None
        pmc = os.path.join(ROOT, "profiles", PMC_FILE)
        if os.path.exists(pmc) and a.nodes_per_rank == NODES_PER_RANK:
            traffic = json.load(open(pmc))["kernels"]["k_tick"]["hbm_bytes"]
            traffic_src = "profiles/%s (rocprofv3 FETCH_SIZE + WRITE_SIZE per launch, same config)" % PMC_FILE
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
            "config": {"workload": "C2 steady-state heartbeat + status ticks (configs[1])",
                       "nodes": fl.total_nodes, "pods": fl.total_nodes * workload.PODS_PER_NODE,
                       "nodes_per_gpu": a.nodes_per_rank, "pods_per_node": workload.PODS_PER_NODE,
                       "cidr": workload.CIDR, "buckets": workload.BUCKETS, "parallelism": "bucket-sharded x%d" % world},
            "tick_api": ("kwok_tick_submit/kwok_tick_collect, tick k+1 queued before tick k is collected"
                         if a.queue else "kwok_tick"),
            "ms_per_step_kwok_tick": dt_sync / a.steps * 1e3,  # the same steps, one blocking kwok_tick each
            "objects_evaluated_per_s": evald / dt,
            "phase_ms_per_tick": {k: v / max(nt, 1) for k, v in phases.items()},
            "host_ms_per_tick": {k: v / max(host_n, 1) for k, v in host_ms.items()},
            "initial_tick_counters": first,
            "setup_s": setup_s,
            "roofline": {"bound": "hbm", "kernel": "k_tick", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "bytes_per_launch": alg_bytes, "avg_launch_ms": kern_ms,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "timing": "HIP events around each k_tick launch (hipExtLaunchKernelGGL), %d ticks" % nt},
        }
        if world == 1 and a.cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.cpu_nodes)
        print(json.dumps(out))
    e.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
