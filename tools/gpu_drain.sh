set -o pipefail
R=$GRAFT_REPO_ROOT
for v in base norel nogjob nowc; do
  lib=$R/kwok_amd/lib/libkwok_engine.so; [ $v != base ] && lib=$R/kwok_amd/lib/var/libkwok_engine_$v.so
  KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=3 KWOK_ENGINE_LIB=$lib timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 3 > gpurun_out/drain_$v.json 2> gpurun_out/drain_$v.err
  echo "$v rc=$? $(grep '^{' gpurun_out/drain_$v.json | cut -c1-120)"
  grep -E "pods-done|block-sum|drained|arrived|reduced|pool-done" gpurun_out/drain_$v.err | tail -6
done
