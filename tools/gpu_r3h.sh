#!/bin/bash
# Round-3 checkpoint H (diagnostics): H2D of page-locked batches after a
# pageable / page-locked 100 MB D2H (the bench's dump_pods between churn steps).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 python tools/h2d_probe.py > $R/gpurun_out/r3h_h2d.txt 2>&1 || exit 2
grep h2d $R/gpurun_out/r3h_h2d.txt
exit 0
