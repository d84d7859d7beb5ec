#!/bin/bash
# A/B of engine builds on one box for the C4 churn ingest: alternating churn-leg
# runs (KWOK_ENGINE_LIB), ingest phase timings (KWOK_INGEST_PROF=1) summarised as
# medians.  Usage: ab_ingest.sh ROUNDS LIB...
R=$GRAFT_REPO_ROOT
N=$1; shift
for i in $(seq $N); do
  for L in "$@"; do
    KWOK_ENGINE_LIB=$L KWOK_INGEST_PROF=1 timeout -k 10 200 python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --roofline-ticks 0 --flap-ticks 0 --churn-ticks 5 > $R/gpurun_out/abi.json 2> $R/gpurun_out/abi.err || { echo "FAIL $L"; tail -5 $R/gpurun_out/abi.err; exit 1; }
    python3 - "$L" $R/gpurun_out/abi.json $R/gpurun_out/abi.err <<'PY'
import json, re, sys, statistics as st, os
d = json.load(open(sys.argv[2]))["churn"]
rows = [tuple(map(float, m)) for m in re.findall(r"route ([\d.]+) ms, records ([\d.]+) ms, flush ([\d.]+) ms", open(sys.argv[3]).read())][-5:]
med = lambda k: st.median(r[k] for r in rows)
print("%-28s churn step %.2f ms ingest %.2f | route %.2f records %.2f flush %.2f" % (os.path.basename(sys.argv[1]), d["median_ms"]["step"], d["median_ms"]["ingest"], med(0), med(1), med(2)))
PY
  done
done
