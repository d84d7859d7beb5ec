#!/bin/bash
# Round-3 diagnostics L: (1) H2D rate of page-locked 96 MB batches per round,
# default and blit-kernel copies (SDMA off), and the churn ingest with SDMA off;
# (2) per-phase stamps of split churn ticks; (3) kernel trace of a churn run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 python tools/h2d_probe.py > $R/gpurun_out/r3l_h2d.txt 2>&1 || { tail $R/gpurun_out/r3l_h2d.txt; exit 2; }
HSA_ENABLE_SDMA=0 timeout -k 10 120 python tools/h2d_probe.py >> $R/gpurun_out/r3l_h2d.txt 2>&1 || exit 3
grep h2d $R/gpurun_out/r3l_h2d.txt
HSA_ENABLE_SDMA=0 KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --churn-ticks 5 --flap-ticks 0 > $R/gpurun_out/r3l_ing.json 2> $R/gpurun_out/r3l_ing.err || exit 4
grep -E "2000000 pod" $R/gpurun_out/r3l_ing.err
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 KWOK_TICK_TRACE_COUNT=3 timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 1 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3l_trace.json 2> $R/gpurun_out/r3l_trace.err || exit 5
grep "kwok trace" $R/gpurun_out/r3l_trace.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r3l -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 3 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3l_prof.json 2>&1 || exit 6
T=$(find $R/gpurun_out/prof_r3l -name 'run_kernel_trace.csv' | head -n 1)
python3 - "$T" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    n = r["Kernel_Name"]
    if any(k in n for k in ("k_tick", "k_pod_jobs", "k_emit", "k_ing_")):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if d > 100 or "k_pod_jobs" in n:
            print("%-40s %9.1f us" % (n.split("(")[0][-40:], d))
PY
exit 0
