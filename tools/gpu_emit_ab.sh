# initial-tick emission A/B: bench's initial_tick line per engine library
# (usage: gpu_emit_ab.sh NAME=LIB[=ENV=V,ENV=V] ...; LIB "-" = the in-tree build)
set -o pipefail
R=$GRAFT_REPO_ROOT
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%=*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*=}
  [ "$lib" = "-" ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  env ${envs//,/ } KWOK_ENGINE_LIB=$lib timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --c2 0 --json-ticks 0 > $R/gpurun_out/eab_$name.json 2> $R/gpurun_out/eab_$name.err || { echo "FAIL $name"; tail -5 $R/gpurun_out/eab_$name.err; exit 1; }
  echo "$name $(python3 $R/tools/last_json.py $R/gpurun_out/eab_$name.json initial_tick | cut -c1-400)"
done
