#!/bin/bash
# heartbeat-once probe: timing, then phase stamps
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 python3 $R/tools/once_probe.py 100 base > $R/gpurun_out/r4b.txt 2> $R/gpurun_out/r4b.err || { tail -5 $R/gpurun_out/r4b.err; exit 2; }
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=8 timeout -k 10 120 python3 $R/tools/once_probe.py 50 trace >> $R/gpurun_out/r4b.txt 2> $R/gpurun_out/r4b_trace.err || { tail -5 $R/gpurun_out/r4b_trace.err; exit 3; }
cat $R/gpurun_out/r4b.txt; grep "kwok trace" $R/gpurun_out/r4b_trace.err
