#!/bin/bash
# ASan/UBSan run of the host codec over golden pod documents and 2000 mutations (CPU only).
set -e
cd "$(dirname "$0")/.."
mkdir -p /tmp/codec_asan
python - <<'PY'
import json, random, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import harness
docs = [json.dumps(harness.pod_doc(e)).encode() for n in harness.TRACES for t in harness.load_trace(n)["ticks"]
        for e in t["pod_events"] if e["op"] == "upsert"]
rng = random.Random(5)
for _ in range(2000):
    b = bytearray(rng.choice(docs))
    for _ in range(rng.randint(1, 6)):
        b[rng.randrange(len(b))] = rng.choice(b'{}[]",:\\0123456789tfnul \x00\xff')
    docs.append(bytes(b)[:rng.randrange(1, len(b) + 1)])
docs.append(b"[" * 5000 + b"]" * 5000)
with open("/tmp/codec_asan/docs.bin", "wb") as f:
    for d in docs:
        f.write(len(d).to_bytes(4, "little") + d)
PY
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -Iinclude -Ikwok_amd/csrc \
  tools/micro/codec_asan.cpp kwok_amd/csrc/codec.cpp kwok_amd/csrc/templates.cpp -o /tmp/codec_asan/t -lpthread
/tmp/codec_asan/t /tmp/codec_asan/docs.bin
