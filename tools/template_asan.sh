#!/bin/bash
# ASan/UBSan run of the host template renderer and compilers over the test
# templates (plus the reference's .tpl files when present) and 3000 mutations (CPU only).
set -e
cd "$(dirname "$0")/.."
mkdir -p /tmp/template_asan
python - <<'PY'
import glob, os, random
srcs = [open(p, "rb").read() for p in glob.glob("tests/templates/*.tpl")]
ref = "/root/reference/pkg/kwok/controllers/templates"
if os.path.isdir(ref):
    srcs += [open(p, "rb").read() for p in glob.glob(ref + "/*.tpl")]
srcs += [b"k: {{ YAML .status 1 }}\n", b"{{ range .spec.containers }}- {{ .name }}\n{{ end }}",
         b"a: [1, {b: 'c''d', e: \"\\u00e9\"}]\n", b"- - - x\n", b"{{ if .a }}{{ else if .b }}{{ else }}{{ end }}"]
rng = random.Random(7)
out = list(srcs)
for _ in range(3000):
    b = bytearray(rng.choice(srcs))
    for _ in range(rng.randint(1, 8)):
        op = rng.random()
        pos = rng.randrange(len(b) + 1)
        if op < 0.4 and len(b):
            b[min(pos, len(b) - 1)] = rng.choice(b'{}[]()|-:"\'.$ \n\t#*&!>%`\\0aZ\x00\xff')
        elif op < 0.7:
            b[pos:pos] = rng.choice([b"{{", b"}}", b"{{ end }}", b"{{ else }}", b"{{-", b"-}}", b"\n  ", b": ", b"- "])
        else:
            del b[pos:pos + rng.randint(1, 20)]
    out.append(bytes(b))
out.append(b"{{ if . }}" * 3000)
out.append(b"- " * 3000 + b"x\n")
out.append(b"[" * 5000 + b"]" * 5000)
with open("/tmp/template_asan/tpl.bin", "wb") as f:
    for d in out:
        f.write(len(d).to_bytes(4, "little") + d)
PY
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -Iinclude -Ikwok_amd/csrc \
  tools/micro/template_asan.cpp kwok_amd/csrc/gotemplate.cpp kwok_amd/csrc/templates.cpp -o /tmp/template_asan/t
/tmp/template_asan/t /tmp/template_asan/tpl.bin
