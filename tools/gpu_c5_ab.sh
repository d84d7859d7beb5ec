# C5 flap A/B per engine library (bench.py with the other legs off: full and heartbeat-once flap lines)
# (usage: gpu_c5_ab.sh NAME=LIB ...; LIB "-" = the in-tree build)
set -o pipefail
R=$GRAFT_REPO_ROOT
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  [ "$lib" = "-" ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$lib timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --once-ticks 1 --emulate-ranks 0 --c2 0 --json-ticks 0 --flap-ticks 6 > $R/gpurun_out/c5ab_$name.json 2> $R/gpurun_out/c5ab_$name.err || { echo "FAIL $name"; tail -5 $R/gpurun_out/c5ab_$name.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/c5ab_$name.json').read().strip().splitlines()[-1])
f=d['flap']; o=(d.get('heartbeat_once') or {}).get('flap') or {}
print('$name', 'flap', round(f['ms_per_step'],4), round(f['ingest_ms'],4), round(f['tick_ms'],4), 'once', o.get('ms_per_step'))"
done
