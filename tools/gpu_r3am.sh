#!/bin/bash
# Round-3 final checkpoint: the full GPU suite, smoke, default bench, kernel trace,
# PMC passes (tools/gpu_full.sh), then the heartbeat-once leg under a kernel trace
# (launch gaps between queued ticks).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_full.sh r3am || exit $?
bash $R/tools/gpu_r3al.sh || exit 9
exit 0
