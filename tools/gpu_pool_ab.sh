#!/bin/bash
# Emulated-ranks churn tick A/B (tools/emul_probe.py: BACK folds 8 ranks' lists) per engine library
# (usage: gpu_pool_ab.sh NAME=LIB ...; LIB "-" = the in-tree build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  [ "$lib" = "-" ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$lib timeout -k 10 300 python3 $R/tools/emul_probe.py --churn-ticks 4 > $R/gpurun_out/pab_$name.json 2> $R/gpurun_out/pab_$name.err || { echo "FAIL $name"; tail -5 $R/gpurun_out/pab_$name.err; exit 1; }
  python3 - "$name" $R/gpurun_out/pab_$name.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = d["churn"]
print("%-6s churn tick %.4f (median %.4f) kernel %.4f pool %.4f exchange %s | steady %.4f" % (
    sys.argv[1], c["tick_ms"], c["median_ms"]["tick"], c["kernel_ms"], c["phase_ms"]["pool"], c["exchange_ms"], d["steady_ms_per_tick"]))
PY
done
