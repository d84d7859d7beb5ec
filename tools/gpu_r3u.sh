#!/bin/bash
# Round-3 checkpoint U: k_emit reads a flat chunk's one or two shape tables from
# a per-wave LDS cache.  GPU suite; A/B against the previous build
# (lib/var/libkwok_engine_head.so), twice each, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3u_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/r3u_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3u_tests.log | head -30; exit $rc; }
for rep in 1 2; do
for v in new head; do
  lib=$R/kwok_amd/lib/var/libkwok_engine_$v.so
  [ $v = new ] && lib=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$lib timeout -k 10 400 python bench.py --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --steps 30 > $R/gpurun_out/r3u_b_${v}_$rep.json 2> $R/gpurun_out/r3u_b_${v}_$rep.err || { tail -5 $R/gpurun_out/r3u_b_${v}_$rep.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['churn']; i=d['initial_tick']; print('%-5s step %.4f | init wall %.3f kern %.3f k_emit %.3f (frac %.3f) | churn kern %.3f k_emit %.3f' % (sys.argv[2], d['ms_per_step'], i['wall_ms'], i['kernel_ms'], i['k_emit_ms'], i['emit_roofline']['frac'], c['kernel_ms'], c['k_emit_ms']))" $R/gpurun_out/r3u_b_${v}_$rep.json $v
done
done
exit 0
