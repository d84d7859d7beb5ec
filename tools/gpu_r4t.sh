#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
KWOK_INGEST_PROF=1 timeout -k 10 300 python3 -u $R/tools/stall_probe.py 40 > $R/gpurun_out/r4t.txt 2> $R/gpurun_out/r4t.err || { tail -5 $R/gpurun_out/r4t.err; exit 4; }
grep step $R/gpurun_out/r4t.txt | awk '{print $4}' | tr '\n' ' '; echo
grep -E "queued in" $R/gpurun_out/r4t.err | sort -t'+' -k1 | awk '{print}' | tail -45 | sort -k6 -n | tail -6
grep -E "queued in" $R/gpurun_out/r4t.err | head -3
