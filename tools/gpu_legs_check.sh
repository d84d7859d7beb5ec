# bench.py with short legs (each secondary leg in its own child process): the legs' lines
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --churn-ticks 4 --flap-ticks 3 --json-ticks 0 "$@" > $R/gpurun_out/legs.json 2> $R/gpurun_out/legs.err || { echo "FAIL"; tail -20 $R/gpurun_out/legs.err; exit 1; }
python3 - <<'PY'
import json, os
d = json.loads(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/legs.json").read().strip().splitlines()[-1])
ho = d["heartbeat_once"]
print("value", d["value"], d["ms_per_step"])
print("main C4", d["churn"]["ms_per_step"], d["churn"]["ingest_ms"], "| once C4", ho["churn"]["ms_per_step"], ho["churn"]["ingest_ms"], "| once step", ho["ms_per_step"])
print("flap", d["flap"]["ms_per_step"], ho["flap"]["ms_per_step"], "| c2", d["c2"]["full_bodies"]["ms_per_step"], d["c2"]["heartbeat_once"]["ms_per_step"])
print("emul", d["emulated_ranks"]["churn"]["tick_ms"], d["emulated_ranks"]["steady_ms_per_tick"])
PY
