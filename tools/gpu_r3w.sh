#!/bin/bash
# Round-3 checkpoint W: k_pod_jobs reads the node flags of its runs' buckets from
# LDS.  GPU suite; kernel trace of a churn run for this build and the previous one
# (lib/var/libkwok_engine_head.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3w_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/r3w_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3w_tests.log | head -30; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for v in new head; do
  lib=$R/kwok_amd/lib/var/libkwok_engine_$v.so
  [ $v = new ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_r3w_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 4 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3w_$v.json 2>&1 || exit 6
  T=$(find $R/gpurun_out/prof_r3w_$v -name 'run_kernel_trace.csv' | head -n 1)
  python3 - "$T" $v <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
d = {}
for r in rows:
    n = r["Kernel_Name"]
    for k in ("k_pod_jobs", "k_emit", "k_tick"):
        if k in n:
            d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
pj = d.get("k_pod_jobs", [])
print(sys.argv[2], "k_pod_jobs initial %.1f us, churn %s" % (pj[0], " ".join("%.1f" % x for x in pj[1:])))
PY
done
exit 0
