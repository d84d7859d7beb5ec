#!/bin/bash
# the enqueue stall with the HIP runtime's log: the gap and what surrounds it
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
AMD_LOG_LEVEL=4 KWOK_INGEST_PROF=1 timeout -k 10 400 python3 -u $R/tools/stall_probe.py 16 > $R/gpurun_out/r4u.txt 2> $R/gpurun_out/r4u.log || { tail -5 $R/gpurun_out/r4u.log; exit 4; }
grep step $R/gpurun_out/r4u.txt | awk '{print $4}' | tr '\n' ' '; echo
wc -l $R/gpurun_out/r4u.log
python3 - $R/gpurun_out/r4u.log <<'PY'
import re, sys
lines = open(sys.argv[1], errors="replace").read().splitlines()
pat = re.compile(r":\s*(\d+)\s*us:")
prev = None
gaps = []
for i, l in enumerate(lines):
    m = pat.search(l)
    if not m:
        continue
    t = int(m.group(1))
    if prev is not None and t - prev[0] > 2500:
        gaps.append((t - prev[0], prev[1], i))
    prev = (t, i)
# only the churn phase: after the first "queued in" line
q0 = next((i for i, l in enumerate(lines) if "queued in" in l), 0)
for g, a, b in sorted(gaps, reverse=True):
    if a < q0:
        continue
    print("gap %.3f ms between lines %d and %d" % (g / 1000, a, b))
    for l in lines[max(a - 8, 0):b + 3]:
        print("   ", l[:230])
    break
PY
gzip -f $R/gpurun_out/r4u.log
