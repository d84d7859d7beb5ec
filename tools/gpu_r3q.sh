#!/bin/bash
# Round-3 checkpoint Q: the pool select takes its words from the prep pass; split ticks
# leave the stream to the streamers. GPU suite, bench, churn kernel trace, tick stamps.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
true
true
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3q_tests.log 2>&1
rc=$?
tail -3 $R/gpurun_out/r3q_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3q_tests.log | head -30; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/r3q_b1.json 2> $R/gpurun_out/r3q_b1.err || { tail -20 $R/gpurun_out/r3q_b1.err; exit 3; }
grep -E "2000000 pod" $R/gpurun_out/r3q_b1.err | head -8
python3 - <<'PY'
import json
for n in ("r3q_b1",):
    d = json.load(open("gpurun_out/%s.json" % n))
    it, ch = d["initial_tick"], d["churn"]
    print(n, "step %.4f" % d["ms_per_step"], "init wall %.3f kern %.3f emit %.3f" % (it["wall_ms"], it["kernel_ms"], it["k_emit_ms"]),
          "churn step %.3f tick %.3f kern %.3f emit %.3f ingest %.2f (median %.2f)" % (ch["ms_per_step"], ch["tick_ms"], ch["kernel_ms"], ch["k_emit_ms"], ch["ingest_ms"], ch["median_ms"]["ingest"]))
    h = d["heartbeat_once"]; print("  hb_once step %.4f kernel %.4f classify %.4f" % (h["ms_per_step"], h["kernel_ms"], h["classify_ms"]))
    f = d["flap"]; print("  flap step %.3f ingest %.3f tick %.3f" % (f["ms_per_step"], f["ingest_ms"], f["tick_ms"]))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r3q -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 3 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3q_prof.json 2>&1 || exit 6
T=$(find $R/gpurun_out/prof_r3q -name 'run_kernel_trace.csv' | head -n 1)
python3 - "$T" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    n = r["Kernel_Name"]
    if any(k in n for k in ("k_tick", "k_pod_jobs", "k_emit")):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if d > 230 or "k_pod_jobs" in n or "k_emit" in n:
            print("%-40s %9.1f us" % (n.split("(")[0][-40:], d))
PY
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 KWOK_TICK_TRACE_COUNT=3 timeout -k 10 300 python $R/bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 1 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3q_trace.json 2> $R/gpurun_out/r3q_trace.err || exit 7
grep "kwok trace" $R/gpurun_out/r3q_trace.err
exit 0
