# C4 churn A/B per engine library (tools/c4_probe.py: ms per step, ingest, tick, kernels)
# (usage: gpu_c4_ab.sh NAME=LIB[=ENV=V,ENV=V] ...; LIB "-" = the in-tree build)
set -o pipefail
R=$GRAFT_REPO_ROOT
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%=*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*=}
  [ "$lib" = "-" ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  env ${envs//,/ } KWOK_ENGINE_LIB=$lib timeout -k 10 300 python3 $R/tools/c4_probe.py --ticks 8 $C4ARGS > $R/gpurun_out/c4ab_$name.json 2> $R/gpurun_out/c4ab_$name.err || { echo "FAIL $name"; tail -5 $R/gpurun_out/c4ab_$name.err; exit 1; }
  echo "$name $(grep '^{' $R/gpurun_out/c4ab_$name.json | cut -c1-260)"
done
