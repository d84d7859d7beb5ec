"""CPU: the C4 churn generator (workload.Churn, BASELINE configs[3]) against
the oracle: every churn tick deletes exactly the marked pods (half with
finalizers, pod_controller.go:155-183), releases their IPs, and the same
number of new pods take exactly the released addresses (ipPool.Get reuses the
usable set before fresh ones, utils.go:83-98)."""
import numpy as np

from kwok_amd import abi, workload
from oracle.oracle import Oracle


def test_churn_generator_on_oracle():
    o, fl, ph = workload.build_engine_fleet(Oracle, 2000, buckets=64)
    n_handles = 64 * fl.cp
    dump = lambda: o.dump_pods(0, n_handles)  # noqa: E731
    now = workload.S0 + 30
    r = o.tick(now, read=False)
    assert r.counters[2] == 20_000
    ch = workload.Churn(ph, np.repeat(fl.node_handles, workload.PODS_PER_NODE), 0, n_handles, 3000, seed=5)
    for t in range(4):
        now += 30
        used, _, _, pip = dump()
        dead = ch.live[:3000].copy()
        released = set(pip[dead].tolist())
        ev, ar = ch.batch(dump, now)
        assert (ev["flags"][:3000] & abi.POD_DELETING).all()
        hs, st, _ = o.ingest_pods_raw(ev, ar)
        ch.applied(hs, st)
        out = o.tick(now)
        c = out.counters
        assert (c["delete"], c["release"], c["pod_patch"], c["alloc"]) == (3000, 3000, 3000, 3000), c
        assert sorted(h for h, _ in out.deletes) == sorted(dead.tolist())
        fin = {int(h): bool(f & abi.POD_HAS_FINALIZERS) for h, f in zip(ev["handle"][:3000], ev["flags"][:3000])}
        assert all(bool(f) == fin[h] for h, f in out.deletes)
        used, phase, _, pip = dump()
        new = hs[3000:]
        assert used[new].all() and (phase[new] == abi.PHASE_RUNNING).all()
        assert set(pip[new].tolist()) == released
        assert int(used.sum()) == 20_000 and c["pods_total"] == 20_000
    o.close()
