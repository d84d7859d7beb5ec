#!/bin/bash
# C4 host stalls: which host allocation / result path they follow (40 steps each)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
run() {
  env "$@" timeout -k 10 300 python3 -u $R/tools/stall_probe.py 40 > $R/gpurun_out/r4r.txt 2> $R/gpurun_out/r4r.err || { tail -5 $R/gpurun_out/r4r.err; exit 4; }
  echo "$@: $(grep step $R/gpurun_out/r4r.txt | awk '{print $4}' | tr '\n' ' ')"
}
run KWOK_X=0
run KWOK_HOST_ALLOC=hip
run KWOK_HOST_THP=0
run KWOK_X=0
run KWOK_HOST_ALLOC=hip
run KWOK_HOST_THP=0
