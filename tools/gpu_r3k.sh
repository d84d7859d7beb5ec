#!/bin/bash
# Round-3 diagnostics K: H2D rate of page-locked 96 MB batches per round
# (alternation check), default and with the blit-kernel copies (SDMA off).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 python tools/h2d_probe.py > $R/gpurun_out/r3k_h2d.txt 2>&1 || { tail $R/gpurun_out/r3k_h2d.txt; exit 2; }
HSA_ENABLE_SDMA=0 timeout -k 10 120 python tools/h2d_probe.py >> $R/gpurun_out/r3k_h2d.txt 2>&1 || exit 3
grep h2d $R/gpurun_out/r3k_h2d.txt
HSA_ENABLE_SDMA=0 KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --churn-ticks 5 --flap-ticks 0 > $R/gpurun_out/r3k_ing.json 2> $R/gpurun_out/r3k_ing.err || exit 4
grep -E "2000000 pod" $R/gpurun_out/r3k_ing.err
exit 0
