#!/bin/bash
# Round-3 diagnostics I: churn ingest phase split (KWOK_INGEST_PROF) and the
# C5 flap ingest split, on the current build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --churn-ticks 5 --flap-ticks 5 > $R/gpurun_out/r3i_b1.json 2> $R/gpurun_out/r3i_b1.err || { tail -20 $R/gpurun_out/r3i_b1.err; exit 3; }
grep -E "kwok ingest|kwok grow" $R/gpurun_out/r3i_b1.err | tail -30
exit 0
