"""debug: the distinct-node-blob scenario of tests/test_emit_paths_gpu.py,
repeated in one process, with the heartbeat region checked in detail"""
import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np
import test_emit_paths_gpu as T
from gpu_common import Driver, new_pods, compare
for rep in range(4):
    for many in (False, True):
        rng = np.random.default_rng(21)
        specs = T.spec_set(rng, 80) if many else None
        kw = dict(cidr="10.0.0.1/8", node_ip="196.168.0.1", buckets=128, node_slots_per_bucket=32, pod_slots_per_bucket=256)
        d = Driver(kw, 21, specs=specs)
        names = ["worker-%05d" % i for i in range(1500)]
        status = [T.node_status(rng, i, rng.random() < 0.8) for i in range(len(names))]
        nh, st = d.nodes(names, managed=1, lockable=1, status=status)
        ev, ar = new_pods(rng, nh, 6000, d.spec, 0.0, None, host_ips=T.HOST_IPS, host_ip_frac=0.2, years=5)
        d.pods(ev, ar)
        for t in range(2):
            eo, oo = d.e.tick(d.now), d.o.tick(d.now)
            d.now += 30
            try:
                compare(eo, oo, "rep %d many %d tick %d" % (rep, many, t))
                print("rep", rep, "many", many, "tick", t, "ok", flush=True)
            except AssertionError as ex:
                print("FAIL", ex, flush=True)
                a = np.frombuffer(eo.arena, np.uint8)
                print("arena", len(eo.arena), "n_init", len(eo.node_inits), "n_pp", len(eo.pod_patches), flush=True)
        d.e.close(); d.o.close()
