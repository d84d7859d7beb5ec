"""GPU: structural fuzzing of the device JSON scanners against the host codec
(json.hip k_json_pods / k_json_nodes vs codec.cpp kwok_decode_pods /
kwok_decode_nodes).  test_json_gpu.py and test_json_nodes_gpu.py mutate bytes;
here the golden documents are mutated as JSON values - a value replaced by
another of any type (null, bool, numbers, strings with escapes and non-ASCII,
empty and nested containers), keys dropped, extra keys, a key repeated ahead
of its original (first-key semantics), key order shuffled, deep nesting - and
written compact or indented, some strings with \\u escapes of plain characters.
Every document: the same status on both sides, and for every decoded one the
same record bytes (pods: name / namespace spans and spec key too; nodes: the
arena with the host's canonical blobs).  Seeded; 8k documents per case.
Reference: pod_controller.go:252-269, 301-343, 404-439; node_controller.go:
206-223, 256-279, 356-391 (what the records carry)."""
import json
import random

import numpy as np
import pytest

import harness
from harness import node_doc, pod_doc
from kwok_amd.codec import Codec
from kwok_amd.engine import Engine, make_config
import test_json_gpu
import test_json_nodes_gpu

pytestmark = pytest.mark.gpu

SCALARS = [None, True, False, 0, 1, -7, 3.5, 1e300, "", "x", "Running", "Pending", "2024-01-01T00:00:00Z",
           "10.0.0.1", "196.168.0.1", "fake", "café", "中文", "tab\there", "q\"uote", "back\\slash"]


def rand_value(rng, depth=0):
    r = rng.random()
    if depth > 3 or r < 0.6:
        return rng.choice(SCALARS)
    if r < 0.8:
        return {rng.choice(["a", "name", "type", "status", "image", "x" * rng.randint(1, 40)]): rand_value(rng, depth + 1)
                for _ in range(rng.randint(0, 3))}
    return [rand_value(rng, depth + 1) for _ in range(rng.randint(0, 3))]


def paths(v, prefix=()):
    """every (container, key) in v"""
    out = []
    if isinstance(v, dict):
        for k, x in v.items():
            out.append((v, k))
            out.extend(paths(x, prefix + (k,)))
    elif isinstance(v, list):
        for i, x in enumerate(v):
            out.append((v, i))
            out.extend(paths(x, prefix + (i,)))
    return out


def mutate(doc, rng):
    """1-3 value-level changes of a copy of doc"""
    d = json.loads(json.dumps(doc))
    for _ in range(rng.randint(1, 3)):
        ps = paths(d)
        if not ps:
            break
        c, k = rng.choice(ps)
        op = rng.random()
        if op < 0.45:
            c[k] = rand_value(rng)
        elif op < 0.65 and isinstance(c, dict):
            del c[k]
        elif op < 0.85 and isinstance(c, dict):
            c[rng.choice(["extra", "zz", "status", "spec", "metadata", "phase", "podIP"])] = rand_value(rng)
        elif isinstance(c[k], (dict, list)):
            c[k] = {"nest": {"nest": [c[k]]}}
    return d


def dup_first(text, rng):
    """a key of some object repeated ahead of it, with another value (first wins)"""
    i = text.find('{"', rng.randrange(max(1, len(text) // 2)))
    if i < 0:
        return text
    return text[:i + 1] + '"%s": %s, ' % (rng.choice(["name", "phase", "spec", "metadata", "status", "annotations"]),
                                          json.dumps(rand_value(rng))) + text[i + 1:]


def escape_some(text, rng):
    """\\u escapes of a few plain letters inside strings (the same decoded text)"""
    out, in_str, esc = [], False, False
    for ch in text:
        if in_str and not esc and ch.isalpha() and ch.isascii() and rng.random() < 0.02:
            out.append("\\u%04x" % ord(ch))
            continue
        out.append(ch)
        if esc:
            esc = False
        elif ch == "\\":
            esc = True
        elif ch == '"':
            in_str = not in_str
    return "".join(out)


def render(d, rng):
    text = json.dumps(d, indent=rng.choice([None, None, 1]), ensure_ascii=rng.random() < 0.5)
    r = rng.random()
    if r < 0.15:
        text = dup_first(text, rng)
    elif r < 0.3:
        text = escape_some(text, rng)
    return text.encode()


def corpus(docs, rng, n):
    out = []
    for _ in range(n):
        d = rng.choice(docs)
        if rng.random() < 0.3:
            d = json.loads(test_json_gpu.scramble(d, rng))
        out.append(render(mutate(d, rng), rng))
    return out


@pytest.fixture(scope="module")
def eng():
    e = Engine(make_config(buckets=64, node_slots_per_bucket=16, pod_slots_per_bucket=128))
    yield e
    e.close()


def golden_pods():
    docs = []
    for name in harness.TRACES:
        for t in harness.load_trace(name)["ticks"]:
            docs += [pod_doc(ev) for ev in t["pod_events"]]
    return docs


def golden_nodes():
    docs = []
    for name in harness.TRACES:
        for t in harness.load_trace(name)["ticks"]:
            docs += [node_doc(ev) for ev in t["node_events"] if ev["op"] != "delete"]
    return docs


@pytest.mark.parametrize("sel", range(len(test_json_gpu.SELECTORS)))
def test_pod_documents_fuzzed(eng, sel):
    rng = random.Random(100 + sel)
    docs = corpus(golden_pods(), rng, 8000)
    codec = Codec(manage_all_nodes=True, **test_json_gpu.SELECTORS[sel])
    _, hs = test_json_gpu.compare(eng, codec, docs, where="fuzzed pods %d" % sel)
    assert (hs == 0).sum() > 100 and (hs != 0).sum() > 100  # both outcomes well represented


@pytest.mark.parametrize("sel", range(len(test_json_nodes_gpu.SELECTORS)))
def test_node_documents_fuzzed(eng, sel):
    rng = random.Random(200 + sel)
    docs = corpus([test_json_nodes_gpu.with_labels(d, rng) for d in golden_nodes()], rng, 8000)
    codec = Codec(**test_json_nodes_gpu.SELECTORS[sel])
    test_json_nodes_gpu.compare(eng, codec, docs, where="fuzzed nodes %d" % sel)
