#!/bin/bash
# Round-3 checkpoint G (diagnostics): H2D of page-locked batches under device
# memory traffic, hipHostMalloc vs huge-page registered buffers; churn A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 python tools/h2d_probe.py > $R/gpurun_out/r3g_h2d.txt 2>&1 || exit 2
KWOK_HOST_ALLOC=hip timeout -k 10 120 python tools/h2d_probe.py >> $R/gpurun_out/r3g_h2d.txt 2>&1 || exit 2
grep h2d $R/gpurun_out/r3g_h2d.txt
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 20 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --churn-ticks 8 > $R/gpurun_out/r3g_b1.json 2> $R/gpurun_out/r3g_b1.err || exit 3
grep "2000000 pod" $R/gpurun_out/r3g_b1.err
exit 0
