#!/bin/bash
# Round-3 checkpoint AA: node ingest partitions on their own cache lines; Use
# checks skipped while no foreign podIP entered the pool.  GPU suite, C5 flap at
# 16 / 4 partition threads, churn-tick stamps, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/raa_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/raa_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/raa_tests.log | head -30; exit $rc; }
for th in 16 4; do
  KWOK_INGEST_THREADS=$th KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --churn-ticks 0 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 8 > $R/gpurun_out/raa_flap$th.json 2> $R/gpurun_out/raa_flap$th.err || exit 2
  grep "9990 node" $R/gpurun_out/raa_flap$th.err | tail -2
  python3 -c "import json; f=json.load(open('$R/gpurun_out/raa_flap$th.json'))['flap']; print('threads $th: step %.3f ingest %.3f tick %.3f' % (f['ms_per_step'], f['ingest_ms'], f['tick_ms']))"
done
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 KWOK_TICK_TRACE_COUNT=3 timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 1 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/raa_trace.json 2> $R/gpurun_out/raa_trace.err || exit 3
grep -E "kwok trace\] chain    (pods-done|arrived|reduced|pool-done|exit)" $R/gpurun_out/raa_trace.err
timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/raa_b.json 2> $R/gpurun_out/raa_b.err || exit 4
python3 -c "import json; d=json.load(open('$R/gpurun_out/raa_b.json')); c=d['churn']; f=d['flap']; print('step %.4f | churn step %.3f kern %.3f ingest %.3f | flap %.3f | init %.3f | once %.4f' % (d['ms_per_step'], c['ms_per_step'], c['kernel_ms'], c['ingest_ms'], f['ms_per_step'], d['initial_tick']['wall_ms'], d['heartbeat_once']['ms_per_step']))"
exit 0
