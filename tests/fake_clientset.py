"""An in-memory clientset for the controller tests: the role client-go's
fake.NewSimpleClientset plays in the reference's unit tests
(node_controller_test.go:38-66, pod_controller_test.go:38-71), with what the
drop-in relies on from a real apiserver:

- every write bumps a global resourceVersion and produces a watch event that
  carries it (the drop-in drops the echoes of its own patches by it);
- a watch first sends an ADDED event per existing object (a watch without
  resourceVersion, as List + Watch), then every change;
- PatchStatus / Patch(status) apply a strategic merge patch: maps merge
  recursively, null deletes a key, lists with a patchMergeKey in corev1
  (conditions and addresses by type, podIPs by ip) merge by that key, every
  other list is replaced; Patch(merge) applies an RFC 7386 merge patch;
- NotFound for a missing object.

deliver="sync" hands each event to the watchers inside the write, BEFORE the
write returns (the echo overtakes the patch's response); deliver="queued" holds
the events until pump() (the response first).  A real apiserver does either.
"""
from __future__ import annotations

import copy
import json

from kwok_amd.controller import NotFound

MERGE_KEYS = {"conditions": "type", "addresses": "type", "podIPs": "ip"}


def smp(dst, patch):
    """strategic merge of patch into dst (both JSON maps)"""
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            smp(dst[k], v)
        elif isinstance(v, list) and k in MERGE_KEYS and isinstance(dst.get(k), list):
            key = MERGE_KEYS[k]
            out = list(dst[k])
            for item in v:
                for i, old in enumerate(out):
                    if isinstance(old, dict) and old.get(key) == item.get(key):
                        m = copy.deepcopy(old)
                        smp(m, item)
                        out[i] = m
                        break
                else:
                    out.append(copy.deepcopy(item))
            dst[k] = out
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def merge_patch(dst, patch):
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            merge_patch(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


class FakeClientset:
    def __init__(self, *objects, deliver="sync"):
        self.rv = 0
        self.uid = 0
        self.store = {"nodes": {}, "pods": {}}
        self.watchers = {"nodes": [], "pods": []}
        self.deliver = deliver
        self.pending = []
        self.calls = []  # (verb, kind, key, body) of every write, in order
        for o in objects:
            self.create(o, record=False)

    # ---- helpers --------------------------------------------------------------
    @staticmethod
    def kind_of(obj):
        return "nodes" if obj.get("kind") == "Node" else "pods"

    @staticmethod
    def key_of(kind, obj):
        md = obj["metadata"]
        return md["name"] if kind == "nodes" else (md.get("namespace", "default"), md["name"])

    def _bump(self, obj):
        self.rv += 1
        obj["metadata"]["resourceVersion"] = str(self.rv)

    def _emit(self, kind, typ, obj):
        if not self.watchers[kind]:  # a watch opened later starts from the current state
            return
        ev = (kind, typ, copy.deepcopy(obj))
        if self.deliver == "sync":
            self._send(ev)
        else:
            self.pending.append(ev)

    def _send(self, ev):
        kind, typ, obj = ev
        for cb, sel in self.watchers[kind]:
            if sel(obj):
                cb(typ, copy.deepcopy(obj))

    def pump(self):
        """deliver="queued": hand the held events to the watchers"""
        while self.pending:
            ev = self.pending.pop(0)
            self._send(ev)

    # ---- client-go surface the drop-in uses -------------------------------------
    def watch(self, kind, cb, label_selector="", field_selector=""):
        def sel(obj):
            if kind == "pods" and field_selector == "spec.nodeName!=":
                if not (obj.get("spec") or {}).get("nodeName"):
                    return False
            if kind == "nodes" and label_selector:
                from kwok_amd.codec import selector_matches
                return selector_matches(label_selector, obj["metadata"].get("labels") or {})
            return True
        self.watchers[kind].append((cb, sel))
        for obj in list(self.store[kind].values()):
            if sel(obj):
                cb("ADDED", copy.deepcopy(obj))

    def get(self, kind, key):
        o = self.store[kind].get(key)
        if o is None:
            raise NotFound("%s %s" % (kind, key))
        return copy.deepcopy(o)

    def list(self, kind):
        return [copy.deepcopy(o) for o in self.store[kind].values()]

    def patch_node_status(self, name, body):
        self.calls.append(("patch_status", "nodes", name, body))
        return self._patch("nodes", name, json.loads(body), smp)

    def patch_pod_status(self, ns, name, body):
        self.calls.append(("patch_status", "pods", (ns, name), body))
        return self._patch("pods", (ns, name), json.loads(body), smp)

    def patch_pod(self, ns, name, body):
        self.calls.append(("patch_merge", "pods", (ns, name), body))
        return self._patch("pods", (ns, name), json.loads(body), merge_patch)

    def _patch(self, kind, key, patch, how):
        o = self.store[kind].get(key)
        if o is None:
            raise NotFound("%s %s" % (kind, key))
        how(o, patch)
        self._bump(o)
        self._emit(kind, "MODIFIED", o)
        return copy.deepcopy(o)

    def delete_pod(self, ns, name):
        self.calls.append(("delete", "pods", (ns, name), None))
        self.delete("pods", (ns, name))

    # ---- what the tests do to the cluster -----------------------------------------
    def create(self, obj, record=True):
        obj = copy.deepcopy(obj)
        kind = self.kind_of(obj)
        key = self.key_of(kind, obj)
        if key in self.store[kind]:
            raise ValueError("exists: %s" % (key,))
        md = obj.setdefault("metadata", {})
        if kind == "pods":
            md.setdefault("namespace", "default")
        if not md.get("uid"):
            self.uid += 1
            md["uid"] = "uid-%06d" % self.uid
        obj.setdefault("status", {})
        self._bump(obj)
        self.store[kind][key] = obj
        self._emit(kind, "ADDED", obj)
        return copy.deepcopy(obj)

    def update(self, obj):
        obj = copy.deepcopy(obj)
        kind = self.kind_of(obj)
        key = self.key_of(kind, obj)
        if key not in self.store[kind]:
            raise NotFound(str(key))
        self._bump(obj)
        self.store[kind][key] = obj
        self._emit(kind, "MODIFIED", obj)
        return copy.deepcopy(obj)

    def delete(self, kind, key):
        o = self.store[kind].pop(key, None)
        if o is None:
            raise NotFound(str(key))
        self._bump(o)
        self._emit(kind, "DELETED", o)
