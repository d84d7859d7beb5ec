"""Host codec throughput: decode N apiserver-shaped Pod / Node JSON documents
(kwok_decode_pods / kwok_decode_nodes) with 1 and T host threads.
Usage: python tools/codec_rate.py [N] [T]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kwok_amd import abi  # noqa: E402
from kwok_amd.codec import Codec  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
T = int(sys.argv[2]) if len(sys.argv) > 2 else os.cpu_count()
ST = "2023-12-31T23:59:00Z"


def pod(i):
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "pod-%08d" % i, "namespace": "default", "uid": "6f1c%028x" % i,
                         "resourceVersion": str(1000 + i), "creationTimestamp": ST,
                         "labels": {"app": "fake-pod", "pod-template-hash": "7d9f8c6b5"},
                         "ownerReferences": [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "fake-pod-7d9f8c6b5",
                                              "uid": "a1b2", "controller": True, "blockOwnerDeletion": True}]},
            "spec": {"nodeName": "node-%07d" % (i // 10), "restartPolicy": "Always", "schedulerName": "default-scheduler",
                     "containers": [{"name": "fake-pod", "image": "fake", "resources": {},
                                     "terminationMessagePath": "/dev/termination-log", "imagePullPolicy": "Always"}],
                     "tolerations": [{"key": "kwok.x-k8s.io/node", "operator": "Exists", "effect": "NoSchedule"}]},
            "status": {"phase": "Running", "hostIP": "196.168.0.1", "podIP": "10.%d.%d.%d" % (i >> 16 & 255, i >> 8 & 255, i & 255),
                       "startTime": ST, "qosClass": "BestEffort",
                       "conditions": [{"lastProbeTime": None, "lastTransitionTime": ST, "status": "True", "type": t}
                                      for t in ("Initialized", "Ready", "ContainersReady")],
                       "containerStatuses": [{"image": "fake", "imageID": "", "lastState": {}, "name": "fake-pod",
                                              "ready": True, "restartCount": 0,
                                              "state": {"running": {"startedAt": ST}}}]}}


def run(codec, docs, threads):
    buf = bytearray()
    offs, lens = [], []
    for d in docs:
        offs.append(len(buf)); lens.append(len(d)); buf += d
    n = len(docs)
    cbuf = C.create_string_buffer(bytes(buf), len(buf))
    oa, la = (C.c_uint64 * n)(*offs), (C.c_uint32 * n)(*lens)
    out, st = (abi.PodDoc * n)(), (C.c_int32 * n)()
    t0 = time.perf_counter()
    bad = codec._lib.kwok_decode_pods(codec._h, cbuf, len(buf), oa, la, n, threads, out, st)
    dt = time.perf_counter() - t0
    assert bad == 0 and all(out[k].ev.flags & abi.POD_CONFORMS for k in range(0, n, 997))
    return dt, len(buf)


docs = [json.dumps(pod(i)).encode() for i in range(N)]
codec = Codec()
res = {"docs": N, "avg_doc_bytes": sum(map(len, docs)) / N}
for th in sorted({1, T}):
    dt, nbytes = run(codec, docs, th)
    res["threads_%d" % th] = {"pods_per_s": N / dt, "MB_per_s": nbytes / dt / 1e6, "s": dt}
print(json.dumps(res))
