#!/bin/bash
# Chunked pod ingest timeline: C4 churn steps at 4 chunks under a kernel +
# memory-copy trace, with the host's per-chunk stamps.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
KWOK_INGEST_CHUNK=524288 KWOK_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/rad_prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --churn-ticks 3 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 0 > $R/gpurun_out/rad_churn.json 2> $R/gpurun_out/rad_churn.err || exit 2
grep "kwok ingest" $R/gpurun_out/rad_churn.err | tail -12
exit 0
