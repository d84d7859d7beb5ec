#!/bin/bash
# Round-3 checkpoint F (diagnostics): H2D rates, node ingest split, chain
# blocks per CU A/B on the dirty / heartbeat-once ticks.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 python tools/h2d_probe.py > $R/gpurun_out/r3f_h2d.txt 2>&1 || exit 2
HSA_ENABLE_SDMA=0 timeout -k 10 120 python tools/h2d_probe.py >> $R/gpurun_out/r3f_h2d.txt 2>&1 || exit 2
cat $R/gpurun_out/r3f_h2d.txt | grep h2d
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 30 --cpu-baseline 0 > $R/gpurun_out/r3f_b1.json 2> $R/gpurun_out/r3f_b1.err || exit 3
KWOK_TICK_BLOCKS_PER_CU=2 timeout -k 10 400 python bench.py --steps 30 --cpu-baseline 0 > $R/gpurun_out/r3f_b2.json 2> $R/gpurun_out/r3f_b2.err || exit 4
HSA_ENABLE_SDMA=0 KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 30 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r3f_b3.json 2> $R/gpurun_out/r3f_b3.err || exit 5
exit 0
