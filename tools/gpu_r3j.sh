#!/bin/bash
# Round-3 checkpoint J: split ticks (k_pod_jobs) - GPU suite, default bench, and
# the churn / initial tick with KWOK_SPLIT=0 (chain-block pod emission) for A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3j_tests.log 2>&1
rc=$?
tail -4 $R/gpurun_out/r3j_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3j_tests.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3j_b1.json 2> $R/gpurun_out/r3j_b1.err || { tail -20 $R/gpurun_out/r3j_b1.err; exit 3; }
KWOK_SPLIT=0 timeout -k 10 400 python bench.py --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3j_b0.json 2> $R/gpurun_out/r3j_b0.err || { tail -20 $R/gpurun_out/r3j_b0.err; exit 4; }
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --churn-ticks 5 --flap-ticks 5 > $R/gpurun_out/r3j_ing.json 2> $R/gpurun_out/r3j_ing.err || { tail -20 $R/gpurun_out/r3j_ing.err; exit 5; }
python3 - <<'PY'
import json
for n in ("r3j_b1", "r3j_b0"):
    d = json.load(open("gpurun_out/%s.json" % n))
    it, ch = d["initial_tick"], d["churn"]
    print(n, "step %.4f" % d["ms_per_step"], "init wall %.3f kern %.3f emit %.3f" % (it["wall_ms"], it["kernel_ms"], it["k_emit_ms"]),
          "churn tick %.3f kern %.3f emit %.3f ingest %.2f" % (ch["tick_ms"], ch["kernel_ms"], ch["k_emit_ms"], ch["ingest_ms"]))
PY
grep -E "kwok ingest" $R/gpurun_out/r3j_ing.err | tail -12
exit 0
