#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
run() {
  env "$@" timeout -k 10 300 python3 -u $R/tools/stall_probe.py 30 > $R/gpurun_out/r4w.txt 2> $R/gpurun_out/r4w.err || { tail -5 $R/gpurun_out/r4w.err; exit 4; }
  echo "$@: $(grep step $R/gpurun_out/r4w.txt | awk '{print $4}' | tr '\n' ' ')"
}
run KWOK_X=0
run KWOK_COPY_WARM=0
run KWOK_X=0
run KWOK_X=0
