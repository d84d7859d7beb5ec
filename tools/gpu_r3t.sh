#!/bin/bash
# Round-3 checkpoint T: two speculative groups, releases merged per bitmap word.
# GPU suite; A/B against the previous kernels (lib/var/libkwok_engine_head.so):
# bench (steady, heartbeat-once, churn) and churn-tick stamps; stamps of the
# timing-only variants (no wc bookkeeping / spec words / Use checks).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3t_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/r3t_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3t_tests.log | head -30; exit $rc; }
for v in new head; do
  lib=$R/kwok_amd/lib/var/libkwok_engine_$v.so
  [ $v = new ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$lib timeout -k 10 400 python bench.py --cpu-baseline 0 --flap-ticks 0 > $R/gpurun_out/r3t_b_$v.json 2> $R/gpurun_out/r3t_b_$v.err || { tail -5 $R/gpurun_out/r3t_b_$v.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['churn']; h=d['heartbeat_once']; i=d['initial_tick']; print('%-5s step %.4f classify %.4f | once %.4f (kern %.4f cls %.4f) | churn step %.3f kern %.3f | init kern %.3f' % (sys.argv[2], d['ms_per_step'], d['state_only']['classify_ms'], h['ms_per_step'], h['kernel_ms'], h['classify_ms'], c['ms_per_step'], c['kernel_ms'], i['kernel_ms']))" $R/gpurun_out/r3t_b_$v.json $v
done
for v in new head nowc nospecw nouse; do
  lib=$R/kwok_amd/lib/var/libkwok_engine_$v.so
  [ $v = new ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$lib KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 KWOK_TICK_TRACE_COUNT=3 timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 1 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3t_$v.json 2> $R/gpurun_out/r3t_$v.err || { tail -5 $R/gpurun_out/r3t_$v.err; exit 4; }
  echo "== $v"; grep -E "kwok trace\] chain    (pods-done|arrived|pool-done)" $R/gpurun_out/r3t_$v.err
done
exit 0
