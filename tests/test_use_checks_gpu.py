"""GPU: the Use checks a tick may skip.  configurePod Uses every
evaluated pod's podIP (pod_controller.go:378-382); the engine skips that check
for pods without an event while no podIP it did not assign entered the pool.
The first cases start in that regime (ticks with Puts in between), then bring
a foreign address in through each path the GPU apply pass flags - a create
with another pod's podIP, an update to another pod's podIP, a Deleted event
releasing an address its pod does not hold - and release the duplicated
address, with fresh and reused allocations after it.  The last case is the
one where a skipped Use shows in the output (ipPool.new skips used addresses,
utils.go:68-81).  Engine and oracle are compared after every tick on every
output and on the full pod state (gpu_common.Driver)."""
import numpy as np
import pytest

from gpu_common import Driver, external_deletes, mark_deleting, new_pods
from kwok_amd import abi

pytestmark = pytest.mark.gpu

KW = dict(cidr="10.0.0.1/24", node_ip="196.168.0.1", buckets=16, node_slots_per_bucket=8, pod_slots_per_bucket=64)


def _pods_with_ip(d, node, ips, handles=None):
    """Pending pods (new, or updates of `handles`) holding the given podIPs"""
    n = len(ips)
    ar = abi.Arena()
    ev = np.zeros(n, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1 if handles is None else handles
    ev["node_handle"] = node
    ev["spec_id"] = d.spec[0] if handles is None else d.spec_of[handles]
    ev["creation_unix"] = 1704067100 if handles is None else d.ctime_of[handles]
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    for i, ip in enumerate(ips):
        ev[i]["pod_ip"] = ar.ref(abi.ip4s(int(ip)))
    return ev, bytes(ar.buf)


def _start(seed):
    d = Driver(KW, seed)
    nodes, st = d.nodes(["node-%d" % i for i in range(3)], 1, 1)
    assert (st == 0).all()
    rng = np.random.default_rng(seed)
    ev, ar = new_pods(rng, nodes, 40, d.spec[:1])
    ev["flags"] &= ~np.uint8(abi.POD_DISREGARD)
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] |= abi.POD_STATUS_NONEMPTY
    d.pods(ev, ar)
    for t in range(3):
        d.tick("start %d" % t)
    # churn with releases, no foreign address yet (the skipped checks must hold)
    idx, _, _, _ = d.live()
    d.pods(*mark_deleting(rng, d, idx[:5]))
    d.tick("churn deletes")
    ev, ar = new_pods(rng, nodes, 5, d.spec[:1])
    ev["flags"] &= ~np.uint8(abi.POD_DISREGARD)
    d.pods(ev, ar)
    d.tick("churn creates")
    d.tick("quiet")
    return d, nodes, rng


def _holder_release_then_get(d, nodes, rng, holder, where):
    """release `holder`'s address (the other holder keeps it), then new pods Get"""
    d.pods(*mark_deleting(rng, d, np.array([holder])))
    d.tick(where + ": release")
    d.tick(where + ": the duplicate re-Used")
    ev, ar = new_pods(rng, nodes, 6, d.spec[:1])
    ev["flags"] &= ~np.uint8(abi.POD_DISREGARD)
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] |= abi.POD_STATUS_NONEMPTY
    d.pods(ev, ar)
    d.tick(where + ": Gets")
    d.tick(where + ": quiet")


@pytest.mark.parametrize("seed", [1, 2])
def test_create_with_another_pods_ip(seed):
    d, nodes, rng = _start(seed)
    idx, _, _, pip = d.live()
    holder = int(idx[3])
    ev, ar = _pods_with_ip(d, nodes[0], [pip[3]])
    d.pods(ev, ar)
    d.tick("duplicate create")
    _holder_release_then_get(d, nodes, rng, holder, "create")


@pytest.mark.parametrize("seed", [3])
def test_update_to_another_pods_ip(seed):
    d, nodes, rng = _start(seed)
    idx, _, _, pip = d.live()
    holder, mover = int(idx[2]), int(idx[7])
    ev, ar = _pods_with_ip(d, -1, [pip[2]], handles=np.array([mover], np.int32))
    d.pods(ev, ar)
    d.tick("duplicate update")
    _holder_release_then_get(d, nodes, rng, holder, "update")


@pytest.mark.parametrize("seed", [4])
def test_deleted_event_releasing_another_pods_ip(seed):
    d, nodes, rng = _start(seed)
    idx, _, _, pip = d.live()
    victim, other = int(idx[4]), int(idx[9])
    ev, ar = external_deletes(d, np.array([other], np.int32))
    # the Deleted event carries the victim's address, not its own pod's
    ar = abi.Arena()
    ev[0]["pod_ip"] = ar.ref(abi.ip4s(int(pip[4])))
    d.pods(ev, bytes(ar.buf))
    d.tick("foreign release")
    d.tick("the victim re-Used")
    ev, ar = new_pods(rng, nodes, 6, d.spec[:1])
    ev["flags"] &= ~np.uint8(abi.POD_DISREGARD)
    ev["phase"] = abi.PHASE_PENDING
    ev["flags"] |= abi.POD_STATUS_NONEMPTY
    d.pods(ev, ar)
    d.tick("Gets after the foreign release")
    assert victim in set(d.live()[0].tolist())


def test_foreign_address_ahead_of_the_cursor_is_used_at_relock():
    """The case where a skipped Use would show: pod A is created with a podIP
    ahead of the fresh cursor on an unmanaged node (not evaluated, so not Used);
    when its node becomes managed, the heartbeat re-lock evaluates A without an
    event of its own and configurePod Uses the address, so ipPool.new skips it
    (utils.go:68-81).  Without the foreign-address flag the engine would skip
    A's Use check and hand the address out again."""
    d = Driver(KW, 5)
    (n0, n1), st = d.nodes(["node-a", "node-b"], np.array([1, 0], np.uint8), 1)
    assert (st == 0).all()
    rng = np.random.default_rng(5)
    ev, ar = new_pods(rng, [n0], 10, d.spec[:1])
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    ev["phase"] = abi.PHASE_PENDING
    d.pods(ev, ar)
    d.tick("ten pods: .1 - .10")
    ahead = abi.ip4("10.0.0.15")
    ev, ar = _pods_with_ip(d, n1, [ahead])
    d.pods(ev, ar)
    for t in range(3):
        d.tick("A on the unmanaged node %d" % t)
    d.nodes(["node-b"], 1, 1)  # now managed: A is evaluated at the re-lock
    d.tick("A Used")
    ev, ar = new_pods(rng, [n0], 10, d.spec[:1])
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    ev["phase"] = abi.PHASE_PENDING
    d.pods(ev, ar)
    d.tick("fresh allocation skips A's address")
    d.tick("quiet")
    idx, _, _, pip = d.live()
    assert (pip == ahead).sum() == 1, "A's address handed out again"
