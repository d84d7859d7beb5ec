"""CPU: the oracle enforces the supported domain of tests/domain_cases.py, and
the domain's string rule agrees with the fixture generator's YAML typing
(tests/golden/gotmpl.py) wherever PyYAML's YAML 1.1 resolvers and yaml.v2's
agree (PyYAML also reads base-60 ints, yaml.v2 does not)."""
import numpy as np
import pytest

import domain_cases
import gotmpl_path  # noqa: F401
import gotmpl
from kwok_amd import abi
from kwok_amd.engine import KwokError
from oracle.oracle import Oracle

KW = dict(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8)


def spec_ok(backend, value):
    try:
        backend.register_pod_spec([("c", value)])
        return True
    except KwokError as e:
        assert e.code == abi.EDOMAIN, value
        return False


def node_info_ok(backend, value):
    ar = abi.Arena()
    ev = np.zeros(1, abi.NODE_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["managed"] = 1
    ev[0]["name"] = ar.ref("n0")
    ev[0]["node_info"][abi.NODEINFO_KEYS.index("kernelVersion")] = ar.ref(value) if value else (0, 0)
    _, st = backend.ingest_nodes_raw(ev, bytes(ar.buf))
    return int(st[0])


def pod_ip_status(backend, ip, field):
    spec = backend.register_pod_spec([("c", "img")])
    ar = abi.Arena()
    ev = np.zeros(1, abi.POD_EVENT_DTYPE)
    ev["op"] = abi.OP_UPSERT
    ev["handle"] = -1
    ev["node_handle"] = -1
    ev["spec_id"] = spec
    ev["flags"] = abi.POD_STATUS_NONEMPTY
    ev[0]["node_name"] = ar.ref("n0")
    ev[0][field] = ar.ref(ip)
    _, st, _ = backend.ingest_pods_raw(ev, bytes(ar.buf))
    return int(st[0])


def check_backend(make):
    """the whole table through one backend (oracle here; the engine in
    test_scale_gpu.py::test_domain_table_engine)"""
    for v, ok, why in domain_cases.STRINGS:
        b = make()
        assert spec_ok(b, v) == ok, (v, why)
        if v:  # an empty nodeInfo value is "" (the template's default applies)
            assert node_info_ok(b, v) == (abi.OK if ok else abi.EDOMAIN), (v, why)
        b.close()
    for ip, ok in domain_cases.IPS:
        for field in ("host_ip", "pod_ip"):
            b = make()
            assert pod_ip_status(b, ip, field) == (abi.OK if ok else abi.EDOMAIN), (ip, field)
            b.close()


def test_oracle_domain_table():
    check_backend(lambda: Oracle(**KW))


@pytest.mark.parametrize("v,ok,why", [c for c in domain_cases.STRINGS if c[0] and c[0][0].isalnum()
                                      and ":" not in c[0] and c[0][-1] != " " and "#" not in c[0]
                                      and '"' not in c[0] and c[0] not in domain_cases.PYYAML_DIFFERS])
def test_string_rule_matches_yaml_typing(v, ok, why):
    """in-domain values come out of YAML -> JSON as the same string; values the
    typing rule rejects come out as something else"""
    got = gotmpl.yaml_to_json("k:  %s \n" % v)
    assert (got == '{"k":%s}' % gotmpl.go_json_string(v)) == ok, (v, got, why)


def test_oracle_rejects_cidr_outside_domain():
    for cidr in ("010.0.0.1/8", "1.2.3.4./8", "fe80::1/64"):
        with pytest.raises(KwokError):
            Oracle(cidr=cidr, **KW)
