"""CPU: the C-ABI library builds for gfx950, loads without a GPU, exports every
symbol include/kwok_engine.h declares, and the Python ABI mirror matches the
header's struct layout (checked against gcc on the header itself)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from kwok_amd import abi, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kwok_engine.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kwok_[a-z_0-9]+)\s*\(", src)) - {"kwok_allgather_fn"})


def test_engine_library_exports_every_declared_symbol():
    lib = engine.load_engine_lib()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert lib.kwok_abi_version() == abi.ABI_VERSION


def test_engine_is_gfx950_code_object():
    blob = open(os.path.join(ROOT, "kwok_amd", "lib", "libkwok_engine.so"), "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_oracle_library_exports():
    from oracle import oracle
    lib = oracle.load()
    for f in declared_functions():
        name = f.replace("kwok_", "kwok_oracle_", 1)
        if f in ("kwok_engine_create", "kwok_engine_destroy"):
            name = name.replace("engine_", "")
        if f in ("kwok_abi_version", "kwok_comm_id", "kwok_finalizer_patch", "kwok_device_outputs",
                 "kwok_host_alloc", "kwok_host_free",  # engine only: page-locked batch buffers
                 "kwok_pack_pod_events",  # host helper of the compact wire form (engine library)
                 "kwok_bucket_of", "kwok_rank_of_bucket", "kwok_profile_enable", "kwok_profile_read", "kwok_profile_host",
                 "kwok_tick_submit", "kwok_tick_collect",  # engine only: queued ticks (the oracle is sequential)
                 "kwok_ingest_pods_packed12_tick",  # engine only: a batch with its tick queued behind it
                 "kwok_read_arena_async", "kwok_read_wait",  # engine only: reads overlapping the next tick
                 "kwok_engine_stats",  # engine only: which tick kernel ran
                 "kwok_spec_key", "kwok_decode_pods_gpu", "kwok_ingest_pods_json",  # the GPU codec (engine library)
                 "kwok_ingest_nodes_json", "kwok_decode_nodes_gpu",
                 "kwok_codec_create", "kwok_codec_destroy", "kwok_codec_last_error", "kwok_selector_matches",
                 "kwok_decode_node", "kwok_decode_pod", "kwok_decode_nodes", "kwok_decode_pods",  # host codec: feeds both, lives in the engine library
                 "kwok_template_render", "kwok_template_last_error", "kwok_pod_template_patch",
                 "kwok_node_template_patch", "kwok_heartbeat_template_patch"):  # host template compiler (engine library)
            continue
        assert hasattr(lib, name), name


STRUCTS = {
    "kwok_node_event": (abi.NodeEvent, ["op", "managed", "lockable", "phase", "name", "addresses", "allocatable",
                                        "capacity", "node_info"]),
    "kwok_pod_event": (abi.PodEvent, ["op", "phase", "flags", "handle", "spec_id", "node_handle", "creation_unix",
                                      "node_name", "host_ip", "pod_ip"]),
    "kwok_pod_rec": (abi.PodRec, ["op", "flags", "spec_id", "target", "creation", "host_ip", "pod_ip"]),
    "kwok_pod_spec": (abi.PodSpec, ["containers", "n_containers", "init_containers", "n_init_containers",
                                    "readiness_gates", "n_readiness_gates"]),
    "kwok_config": (abi.Config, ["abi_version", "cidr", "node_ip", "start_time_unix", "enable_cni",
                                 "custom_templates", "buckets", "node_slots_per_bucket", "pod_slots_per_bucket",
                                 "max_pod_specs", "rank", "world_size", "device", "comm_id", "allgather",
                                 "allgather_user", "pod_handle_stride", "flags", "pod_status_template",
                                 "node_init_template", "node_heartbeat_template"]),
    "kwok_tick_result": (abi.TickResult, ["n_heartbeat", "heartbeat_len", "heartbeat_stride", "n_node_init",
                                          "n_pod_patch", "n_delete", "heartbeat_epoch", "arena_bytes", "counters",
                                          "local_counters"]),
    "kwok_outputs": (abi.Outputs, ["heartbeat_nodes", "heartbeat_off", "node_init_nodes", "node_init_off",
                                   "node_init_len", "pod_patch_pods", "pod_patch_off", "pod_patch_len",
                                   "delete_pods", "delete_has_finalizers", "arena", "arena_cap", "flags",
                                   "arena_shift", "arena_copied"]),
    "kwok_codec_config": (abi.CodecConfig, ["manage_all_nodes", "manage_nodes_with_annotation_selector",
                                            "manage_nodes_with_label_selector",
                                            "disregard_status_with_annotation_selector",
                                            "disregard_status_with_label_selector"]),
    "kwok_pod_doc": (abi.PodDoc, ["ev", "name", "namespace_", "n_containers", "n_init_containers",
                                  "n_readiness_gates", "containers", "init_containers", "readiness_gates"]),
    "kwok_device_view": (abi.DeviceView, ["arena", "heartbeat_nodes", "pod_patch_pods", "pod_patch_off",
                                          "pod_patch_len", "stream"]),
}


def test_struct_layout_matches_header():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HEADER, "int main(void){"]
    for cname, (_, fields) in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in fields:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "l.c")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-o", os.path.join(d, "l"), src])
        out = subprocess.check_output([os.path.join(d, "l")], text=True)
    got = dict(l.split() for l in out.strip().splitlines())
    for cname, (st, fields) in STRUCTS.items():
        assert int(got[cname]) == C.sizeof(st), cname
        for f in fields:
            assert int(got["%s.%s" % (cname, f)]) == getattr(st, f).offset, (cname, f)
    assert abi.NODE_EVENT_DTYPE.itemsize == C.sizeof(abi.NodeEvent)
    assert abi.POD_EVENT_DTYPE.itemsize == C.sizeof(abi.PodEvent)
    assert abi.POD_REC_DTYPE.itemsize == C.sizeof(abi.PodRec) == 20


def test_bucket_helpers():
    lib = engine.load_engine_lib()
    for name in ["node-0000000", "node0", "kwok-node-0", "x"]:
        b = name.encode()
        assert lib.kwok_bucket_of(b, len(b), 4096) == abi.fnv1a32(name) & 4095
    assert [lib.kwok_rank_of_bucket(b, 4096, 8) for b in (0, 511, 512, 4095)] == [0, 0, 1, 7]


def test_finalizer_patch_constant():
    # pod_controller.go:45
    assert engine.finalizer_patch() == b'{"metadata":{"finalizers":null}}'


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(engine.KwokError):
        engine.Engine(buckets=16, node_slots_per_bucket=4, pod_slots_per_bucket=8)


def test_profile_enums_match_python_mirrors():
    """The diagnostic buffers Engine passes are sized from these tuples: they
    must list exactly the KWOK_T_* / KWOK_H_* entries of the header, in order."""
    from kwok_amd.engine import Engine
    hdr = open(os.path.join(ROOT, "include", "kwok_engine.h")).read()
    for prefix, names in (("KWOK_T_", Engine.PHASES), ("KWOK_H_", Engine.HOST), ("KWOK_STAT_", Engine.STATS)):
        body = re.search(r"enum\s*\{\s*(%s\w+[^}]*)\}" % prefix, hdr).group(1)
        ents = [re.sub(r"\s*=.*", "", x).strip() for x in re.sub(r"/\*.*?\*/", "", body).split(",")]
        ents = [x for x in ents if x]
        assert ents[-1] == prefix + "COUNT"
        assert [x[len(prefix):].lower() for x in ents[:-1]] == list(names)


def test_compact_readout_oracle():
    """KWOK_READ_HEARTBEAT_ONCE: one heartbeat body, then the patch region at
    offsets shifted by arena_shift - the same patches as the full copy"""
    import harness
    from oracle.oracle import Oracle
    fx = harness.load_trace("specs")
    o = Oracle(harness.config_for(fx))
    seen = []
    harness.replay(fx, o, on_tick=lambda ti, t, out: seen.append(ti))
    full = o.read_outputs()
    once = o.read_outputs(heartbeat_once=True)
    assert once.node_inits == full.node_inits and once.pod_patches == full.pod_patches
    assert once.heartbeat_body(0) == full.heartbeat_body(0) and len(full.heartbeat_nodes) > 1
    assert len(once.arena) == len(full.arena) - (len(full.heartbeat_nodes) - 1) * full.heartbeat_len


def test_shim_read_sequence_oracle():
    """The Go drop-in's read sequence (lists without an arena, kwok_read_arena of
    one heartbeat body, the patches in bounded pieces) over the oracle's ABI:
    the same bytes as the one-copy read (gpu_common.shim_read_check, which the
    GPU test runs on the 1M x 10M initial tick)"""
    import harness
    from gpu_common import shim_read_check
    from oracle.oracle import Oracle
    fx = harness.load_trace("specs")
    o = Oracle(harness.config_for(fx))
    got = []
    harness.replay(fx, o, on_tick=lambda ti, t, out: got.append(shim_read_check(o, o.read_arrays(), o.last, 2048)))
    assert sum(p for p, _ in got) > 4 and sum(n for _, n in got) > 4096, got
    with pytest.raises(engine.KwokError):  # outside the arena
        o.read_arena(o.last.arena_bytes - 4, 8)
    o.close()
