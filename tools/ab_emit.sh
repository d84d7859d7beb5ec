#!/bin/bash
# A/B of k_emit variants: initial-tick and churn-tick k_emit times from bench.py.
# Usage: ab_emit.sh "NAME=LIB[:ENV=V]" ...   (LIB "-" = the in-tree build)
R=$GRAFT_REPO_ROOT
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*:}
  [ "$lib" = "-" ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  env KWOK_ENGINE_LIB=$lib $envs timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --roofline-ticks 5 --churn-ticks 3 --flap-ticks 0 > $R/gpurun_out/ab_$name.json 2> $R/gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -5 $R/gpurun_out/ab_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[2])); i=d['initial_tick']; c=d['churn']; print('%-10s initial k_emit %.3f ms (frac %.3f)  churn k_emit %.3f ms  step %.1f us' % (sys.argv[1], i['k_emit_ms'], i['emit_roofline']['frac'], c['k_emit_ms'], d['ms_per_step']*1e3))" $name $R/gpurun_out/ab_$name.json
done
