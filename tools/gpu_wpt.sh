set -o pipefail
R=$GRAFT_REPO_ROOT
for v in base wpt2 wpt1 base wpt2 wpt1; do
  lib=$R/kwok_amd/lib/libkwok_engine.so; [ $v != base ] && lib=$R/kwok_amd/lib/var/libkwok_engine_$v.so
  KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=3 KWOK_ENGINE_LIB=$lib timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 4 > gpurun_out/wpt_$v.json 2> gpurun_out/wpt_$v.err || { tail -5 gpurun_out/wpt_$v.err; exit 1; }
  echo "$v $(grep '^{' gpurun_out/wpt_$v.json | cut -c1-200)"
  grep -E "reduced|pool-done|B-prepped|B-selected|pool-folded" gpurun_out/wpt_$v.err
done
