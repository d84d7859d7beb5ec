#!/bin/bash
# A/B of engine builds on one box for the C5 flap leg (node ingest + tick),
# alternating runs; prints the node-ingest phase medians (KWOK_INGEST_PROF=1).
# Usage: ab_flap.sh ROUNDS LIB...
R=$GRAFT_REPO_ROOT
N=$1; shift
for i in $(seq $N); do
  for L in "$@"; do
    KWOK_ENGINE_LIB=$L KWOK_INGEST_PROF=1 timeout -k 10 200 python3 $R/bench.py --steps 3 --warmup 2 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 5 > $R/gpurun_out/abf.json 2> $R/gpurun_out/abf.err || { echo "FAIL $L"; tail -5 $R/gpurun_out/abf.err; exit 1; }
    python3 - "$L" $R/gpurun_out/abf.json $R/gpurun_out/abf.err <<'PY'
import json, re, sys, statistics as st, os
d = json.load(open(sys.argv[2]))["flap"]
rows = [float(m) for m in re.findall(r"node records: records ([\d.]+) ms", open(sys.argv[3]).read())][-5:]
print("%-28s flap step %.2f ms ingest %.2f tick %.3f | node records %.2f ms (median)" % (os.path.basename(sys.argv[1]), d["ms_per_step"], d["ingest_ms"], d["tick_ms"], st.median(rows)))
PY
  done
done
