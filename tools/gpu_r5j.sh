#!/bin/bash
# kernel trace of the C5 flap steps (node ingest on the GPU + tick)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r5j -o run -- python3 $R/bench.py --steps 5 --warmup 2 --roofline-ticks 0 --cpu-baseline 0 --churn-ticks 0 --once-ticks 0 --emulate-ranks 0 --flap-ticks 10 > $R/gpurun_out/r5j.json 2> $R/gpurun_out/r5j.err || { tail -5 $R/gpurun_out/r5j.err; exit 4; }
K=$(find $R/gpurun_out/r5j -name 'run_kernel_trace.csv' | head -n 1)
M=$(find $R/gpurun_out/r5j -name 'run_memory_copy_trace.csv' | head -n 1)
python3 - "$K" "$M" <<'PY'
import csv, sys
ev = []
for r in csv.DictReader(open(sys.argv[1])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]))
for r in csv.DictReader(open(sys.argv[2])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")[:20] + " %s B" % r.get("Size", "")))
ev.sort()
# the last flap step: from the last k_nd_prep on
i = max(k for k, e in enumerate(ev) if "k_nd_prep" in e[2])
t0 = ev[i][0]
for s, e, n in ev[i:i + 40]:
    print("%8.1f %7.1f us  %s" % ((s - t0) / 1e3, (e - s) / 1e3, n))
PY
