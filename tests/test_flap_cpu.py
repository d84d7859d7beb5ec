"""CPU: the C5 flap generator (workload.Flap, BASELINE configs[4]) against the
oracle under partial management: Size() stays the managed count, every
flapped node is locked again and gets its init patch, heartbeats go to the
managed nodes only, and pods of unmanaged nodes are never evaluated."""
from kwok_amd import workload
from oracle.oracle import Oracle


def test_flap_generator_on_oracle():
    o, fl, ph = workload.build_engine_fleet(Oracle, 4000, buckets=64, managed_frac=0.5, lockable_frac=0.999, seed=3)
    managed = int(fl.node_events["managed"].sum())
    lockable_managed = int((fl.node_events["managed"] & fl.node_events["lockable"]).sum())
    assert 1800 < managed < 2200
    now = workload.S0 + 30
    r = o.tick(now, read=False)
    c = r.counters
    assert c[0] == managed and c[8] == managed           # heartbeat, nodes_managed
    assert c[1] == lockable_managed                      # node inits: managed and lockable
    assert c[2] == 10 * managed and c[6] == 10 * managed  # pods of managed nodes only
    f = workload.Flap(fl, 0.01, seed=4)
    for t in range(3):
        now += 30
        ev, ar = f.batch()
        _, st = o.ingest_nodes_raw(ev, ar)
        assert (st == 0).all()
        assert o.node_size() == managed
        r = o.tick(now, read=False)
        c = r.counters
        assert c[0] == managed and c[8] == managed
        assert c[1] == f.k and c[2] == 0 and c[3] == 0   # the flapped nodes re-initialised, no pod patch
    o.close()
