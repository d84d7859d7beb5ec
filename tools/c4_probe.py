"""The bench's C4 churn leg alone (1M x 10M fleet, 1M + 1M records per tick,
kwok_pod_rec12 by default) for kernel traces: tools/gpu_c4.sh runs it under
rocprofv3 and prints the timeline of the last step.

usage: c4_probe.py [--ticks 3] [--wire 12|20|0] [--once] [--steady N]  (--once: a KWOK_CFG_HEARTBEAT_ONCE engine;
--steady: N queued steady ticks before the churn, as bench.py's legs)"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kwok_amd import engine as keng, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ticks", type=int, default=3)
    ap.add_argument("--wire", type=int, default=12)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--once", action="store_true")
    ap.add_argument("--steady", type=int, default=0)
    ap.add_argument("--together", action="store_true", help="kwok_ingest_pods_packed12_tick (the tick behind the batch)")
    a = ap.parse_args()
    e, fl, pods = workload.build_engine_fleet(keng.Engine, a.nodes, heartbeat_once=a.once)
    now = workload.S0 + 30
    e.tick(now, read=False)
    if a.steady:
        _, _, now = bench.steady_queued(e, now, a.steady, 3)
    now += 30
    _, _, c = bench.churn_leg(e, fl, pods, now, a.ticks, a.nodes, packed=a.wire, once=a.once,
                              together=a.together)
    e.close()
    print(json.dumps({k: c[k] for k in ("ms_per_step", "ingest_ms", "tick_ms", "median_ms", "kernel_ms", "roofline",
                                        "phase_ms")}), flush=True)


if __name__ == "__main__":
    main()
