#!/bin/bash
# Round-3 checkpoint M: in-place pod batch reads (kwok_host_alloc buffers) and
# the pipelined classify rows - GPU suite, bench, ingest A/B, churn-tick trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3m_tests.log 2>&1
rc=$?
tail -3 $R/gpurun_out/r3m_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3m_tests.log | head -30; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/r3m_b1.json 2> $R/gpurun_out/r3m_b1.err || { tail -20 $R/gpurun_out/r3m_b1.err; exit 3; }
grep -E "2000000 pod|9990 node" $R/gpurun_out/r3m_b1.err | head -8
KWOK_INGEST_ZC=0 KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --churn-ticks 5 --flap-ticks 0 > $R/gpurun_out/r3m_zc0.json 2> $R/gpurun_out/r3m_zc0.err || exit 4
grep -E "2000000 pod" $R/gpurun_out/r3m_zc0.err
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 KWOK_TICK_TRACE_COUNT=3 timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 1 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3m_trace.json 2> $R/gpurun_out/r3m_trace.err || exit 5
grep "kwok trace" $R/gpurun_out/r3m_trace.err
python3 - <<'PY'
import json
for n in ("r3m_b1", "r3m_zc0"):
    d = json.load(open("gpurun_out/%s.json" % n))
    it, ch = d["initial_tick"], d["churn"]
    print(n, "step %.4f" % d["ms_per_step"], "init wall %.3f kern %.3f emit %.3f" % (it["wall_ms"], it["kernel_ms"], it["k_emit_ms"]),
          "churn step %.3f tick %.3f kern %.3f emit %.3f ingest %.2f (median %.2f)" % (ch["ms_per_step"], ch["tick_ms"], ch["kernel_ms"], ch["k_emit_ms"], ch["ingest_ms"], ch["median_ms"]["ingest"]))
    if "heartbeat_once" in d:
        h = d["heartbeat_once"]; print("  hb_once step %.4f kernel %.4f classify %.4f" % (h["ms_per_step"], h["kernel_ms"], h["classify_ms"]))
    if "flap" in d:
        f = d["flap"]; print("  flap step %.3f ingest %.3f tick %.3f" % (f["ms_per_step"], f["ingest_ms"], f["tick_ms"]))
PY
exit 0
