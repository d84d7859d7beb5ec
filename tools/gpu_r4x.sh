#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
run() {
  env "$@" timeout -k 10 300 python3 -u $R/tools/stall_probe.py 16 > $R/gpurun_out/r4x.txt 2> $R/gpurun_out/r4x.err || { tail -5 $R/gpurun_out/r4x.err; exit 4; }
  echo "$@: $(grep step $R/gpurun_out/r4x.txt | awk '{print $4}' | tail -12 | tr '\n' ' ')"
}
for C in 1048576 700000 500000 350000 1048576 700000 500000 350000; do run KWOK_INGEST_CHUNK=$C; done
