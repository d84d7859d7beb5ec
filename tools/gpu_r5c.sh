#!/bin/bash
# SQ counters of the heartbeat-once k_tick (where its 36 us go)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $R/gpurun_out/r5c -o run -- python3 $R/tools/once_probe.py 20 pmc > $R/gpurun_out/r5c.txt 2>&1 || { tail -5 $R/gpurun_out/r5c.txt; exit 4; }
C=$(find $R/gpurun_out/r5c -name 'run_counter_collection.csv' | head -n 1)
python3 - "$C" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_tick" in r.get("Kernel_Name", "")]
by = collections.defaultdict(lambda: collections.defaultdict(float))
ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-20:]
for r in rows:
    if int(r["Dispatch_Id"]) in ids:
        by[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
for k, v in sorted(by.items()):
    print("%-22s %14.0f per dispatch (mean of %d)" % (k, sum(v.values()) / len(v), len(v)))
PY
