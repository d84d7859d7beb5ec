#!/bin/bash
# Round-3 checkpoint R: quiet ticks (Use checks for event pods only), the
# same-interval echo golden trace; GPU suite, bench, A/B KWOK_QUIET=0, churn
# tick stamps with KWOK_SPLIT=0 (classification cost of the split bookkeeping).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3r_tests.log 2>&1
rc=$?
tail -3 $R/gpurun_out/r3r_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3r_tests.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/r3r_b1.json 2> $R/gpurun_out/r3r_b1.err || { tail -20 $R/gpurun_out/r3r_b1.err; exit 3; }
KWOK_QUIET=0 timeout -k 10 400 python bench.py --cpu-baseline 0 --churn-ticks 0 --flap-ticks 0 > $R/gpurun_out/r3r_q0.json 2> $R/gpurun_out/r3r_q0.err || { tail -20 $R/gpurun_out/r3r_q0.err; exit 4; }
python3 - <<'PY'
import json
for n in ("r3r_b1", "r3r_q0"):
    d = json.load(open("gpurun_out/%s.json" % n))
    it = d["initial_tick"]
    print(n, "step %.4f" % d["ms_per_step"], "k_tick %.4f classify %.4f" % (d["roofline"]["avg_launch_ms"], d["state_only"]["classify_ms"]),
          "init wall %.3f kern %.3f emit %.3f" % (it["wall_ms"], it["kernel_ms"], it["k_emit_ms"]))
    if "churn" in d:
        ch = d["churn"]; print("  churn step %.3f tick %.3f kern %.3f ingest %.2f" % (ch["ms_per_step"], ch["tick_ms"], ch["kernel_ms"], ch["ingest_ms"]))
    h = d["heartbeat_once"]; print("  hb_once step %.4f kernel %.4f classify %.4f" % (h["ms_per_step"], h["kernel_ms"], h["classify_ms"]))
    if "flap" in d:
        f = d["flap"]; print("  flap step %.3f ingest %.3f tick %.3f" % (f["ms_per_step"], f["ingest_ms"], f["tick_ms"]))
PY
KWOK_SPLIT=0 KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 KWOK_TICK_TRACE_COUNT=3 timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 1 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3r_trace.json 2> $R/gpurun_out/r3r_trace.err || exit 7
grep "kwok trace" $R/gpurun_out/r3r_trace.err
exit 0
