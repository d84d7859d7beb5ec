#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
KWOK_INGEST_PROF=1 timeout -k 10 300 python3 -u $R/tools/stall_probe.py 30 > $R/gpurun_out/r4p.txt 2> $R/gpurun_out/r4p.err || { tail -5 $R/gpurun_out/r4p.err; exit 4; }
grep step $R/gpurun_out/r4p.txt | awk '{print $2, $4}' | tr '\n' ' '; echo
grep -E "enqueue \(|wait for its prep|records at \+[2-9]" $R/gpurun_out/r4p.err | head -20
