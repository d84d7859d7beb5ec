#!/bin/bash
# C4 enqueue stalls (an SDMA copy submission holding the host ~6 ms): A/B of copy placement
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
run() {
  env "$@" timeout -k 10 300 python3 -u $R/tools/stall_probe.py 30 > $R/gpurun_out/r4v.txt 2> $R/gpurun_out/r4v.err || { tail -5 $R/gpurun_out/r4v.err; exit 4; }
  echo "$@: $(grep step $R/gpurun_out/r4v.txt | awk '{print $4}' | tr '\n' ' ')"
}
run KWOK_X=0
run KWOK_INGEST_RS=0
run HSA_ENABLE_SDMA=0
run KWOK_INGEST_RESULTS_KERNEL=1
run KWOK_X=0
run KWOK_INGEST_RS=0
run HSA_ENABLE_SDMA=0
run KWOK_INGEST_RESULTS_KERNEL=1
