#!/bin/bash
# Round-3 diagnostics S: churn-tick phase stamps of timing-only variants
# (tools/build_variant.sh): the classification cost of the releases, the
# split bookkeeping, the spec words and the Use checks.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for v in base norel nowc nospecw nouse; do
  lib=$R/kwok_amd/lib/var/libkwok_engine_$v.so
  [ $v = base ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$lib KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 KWOK_TICK_TRACE_COUNT=3 timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 1 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3s_$v.json 2> $R/gpurun_out/r3s_$v.err || { tail -5 $R/gpurun_out/r3s_$v.err; exit 3; }
  echo "== $v"; grep -E "kwok trace\] chain    (pods-done|arrived|reduced|pool-folded|pool-done|exit)" $R/gpurun_out/r3s_$v.err
done
exit 0
