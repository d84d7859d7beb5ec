#!/bin/bash
# the stall probe under a HIP API + memory copy trace: the calls that hold the host in a stalled step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
KWOK_INGEST_PROF=1 timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r4o -o run -- python3 -u $R/tools/stall_probe.py 40 > $R/gpurun_out/r4o.txt 2> $R/gpurun_out/r4o.err || { tail -5 $R/gpurun_out/r4o.err; exit 5; }
grep step $R/gpurun_out/r4o.txt | awk '{print $2, $4}' | tr '\n' ' '; echo
A=$(find $R/gpurun_out/r4o -name 'run_hip_api_trace.csv' | head -n 1)
python3 - "$A" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# calls after the fleet is built: from the first hipMemcpyAsync of an ingest onward, longer than 2 ms
long = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Function"], int(r["Start_Timestamp"]), i) for i, r in enumerate(rows)]
t_end = int(rows[-1]["End_Timestamp"])
for d, f, s, i in long:
    if d > 2_000_000 and f not in ("hipStreamSynchronize",) and s > t_end - 30e9:
        ctx = [rows[j]["Function"] for j in range(max(0, i - 6), i)]
        print("%8.3f ms  %-24s  @%.3f s before end; before it: %s" % (d / 1e6, f, (t_end - s) / 1e9, " ".join(ctx)))
PY
