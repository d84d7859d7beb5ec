#!/bin/bash
# HIP API trace of the churn leg: which call holds the host for milliseconds in a stalled step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
KWOK_INGEST_PROF=1 timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r4m -o run -- python3 $R/bench.py --steps 5 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --churn-ticks 8 > $R/gpurun_out/r4m_churn.json 2> $R/gpurun_out/r4m_churn.err || { tail -5 $R/gpurun_out/r4m_churn.err; exit 5; }
python3 -c "import json; d=json.load(open('$R/gpurun_out/r4m_churn.json')); c=d['churn']; print('churn', c['ms_per_step'], c['median_ms'], c['steps_ms'])"
A=$(find $R/gpurun_out/r4m -name 'run_hip_api_trace.csv' | head -n 1)
python3 - "$A" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
long = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Function"], r["Start_Timestamp"]) for r in rows]
long.sort(reverse=True)
for d, f, s in long[:25]:
    print("%9.3f ms  %s  @%s" % (d / 1e6, f, s))
PY
