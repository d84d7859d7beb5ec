#!/bin/bash
# Heartbeat-once tick, phase stamps (KWOK_TICK_TRACE) and chain blocks per CU A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
B="--steps 40 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 1"
for V in 2 1; do
  KWOK_TICK_BLOCKS_PER_CU=$V timeout -k 10 240 python3 $R/bench.py $B > $R/gpurun_out/r4a_bpc$V.json 2> $R/gpurun_out/r4a_bpc$V.err || { tail -5 $R/gpurun_out/r4a_bpc$V.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['heartbeat_once']; print('bpc', sys.argv[2], d['ms_per_step'], d['kernel_ms'], d['classify_ms'])" $R/gpurun_out/r4a_bpc$V.json $V
done
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=8 timeout -k 10 240 python3 $R/bench.py $B > $R/gpurun_out/r4a_trace.json 2> $R/gpurun_out/r4a_trace.err || { tail -5 $R/gpurun_out/r4a_trace.err; exit 3; }
grep "kwok trace" $R/gpurun_out/r4a_trace.err
exit 0
