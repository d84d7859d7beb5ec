#!/bin/bash
# Round-3 diagnostics Y: C5 node ingest at 4 / 8 / 16 partition threads; the
# initial tick's phase stamps (1M x 10M).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for th in 4 8 16; do
  KWOK_INGEST_THREADS=$th KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --churn-ticks 0 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 8 > $R/gpurun_out/r3y_flap$th.json 2> $R/gpurun_out/r3y_flap$th.err || exit 2
  grep "9990 node" $R/gpurun_out/r3y_flap$th.err | tail -2
  python3 -c "import json; f=json.load(open('$R/gpurun_out/r3y_flap$th.json'))['flap']; print('threads $th: step %.3f ingest %.3f tick %.3f' % (f['ms_per_step'], f['ingest_ms'], f['tick_ms']))"
done
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=0 KWOK_TICK_TRACE_COUNT=1 timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3y_trace_init.json 2> $R/gpurun_out/r3y_trace_init.err || exit 3
grep "kwok trace" $R/gpurun_out/r3y_trace_init.err
exit 0
