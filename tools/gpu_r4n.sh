#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
KWOK_INGEST_PROF=1 timeout -k 10 300 python3 -u $R/tools/stall_probe.py 30 > $R/gpurun_out/r4n_spin.txt 2> $R/gpurun_out/r4n_spin.err || { tail -5 $R/gpurun_out/r4n_spin.err; exit 4; }
cat $R/gpurun_out/r4n_spin.txt
KWOK_SYNC=block timeout -k 10 300 python3 -u $R/tools/stall_probe.py 20 > $R/gpurun_out/r4n_block.txt 2> $R/gpurun_out/r4n_block.err || { tail -5 $R/gpurun_out/r4n_block.err; exit 5; }
cat $R/gpurun_out/r4n_block.txt
grep -B1 -A2 "chunk 1: 750000 records at +[2-9]" $R/gpurun_out/r4n_spin.err | head -20
