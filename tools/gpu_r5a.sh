#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 -u $R/tools/once_probe.py 100 plain > $R/gpurun_out/r5a.txt 2> $R/gpurun_out/r5a.err || { tail -5 $R/gpurun_out/r5a.err; exit 4; }
KWOK_TICK_TRACE=1 timeout -k 10 300 python3 -u $R/tools/once_probe.py 50 trace >> $R/gpurun_out/r5a.txt 2>> $R/gpurun_out/r5a.err || { tail -5 $R/gpurun_out/r5a.err; exit 5; }
cat $R/gpurun_out/r5a.txt; grep -A30 "kwok trace" $R/gpurun_out/r5a.err | head -40
