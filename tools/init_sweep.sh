#!/bin/bash
# Chain-block count sweep: the initial 1M x 10M tick (k_tick + k_emit), the
# steady tick and the churn tick per setting, alternating settings over rounds.
# Usage: init_sweep.sh ROUNDS "ENV..." ...
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
N=$1; shift
for i in $(seq $N); do
  for S in "$@"; do
    env $S timeout -k 10 150 python3 $R/bench.py --steps 100 --warmup 3 --cpu-baseline 0 --roofline-ticks 20 --churn-ticks 3 --flap-ticks 0 > $R/gpurun_out/isw.json 2>/dev/null || { echo "FAIL $S"; exit 1; }
    python3 - "$S" $R/gpurun_out/isw.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); it = d["initial_tick"]; p = d["phase_ms_per_tick"]; c = d["churn"]
print("%-34s init wall %.2f kern %.2f emit %.2f | steady step %.1f us k_tick %.1f classify %.1f | churn tick %.2f ms" % (
    sys.argv[1], it["wall_ms"], it["kernel_ms"], it["k_emit_ms"], d["ms_per_step"] * 1e3, p["kernel"] * 1e3,
    p["classify"] * 1e3, c["median_ms"]["tick"]))
PY
  done
done
