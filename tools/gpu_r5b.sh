#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
: > $R/gpurun_out/r5b.txt
for V in def prev def prev def prev; do
  L=$R/kwok_amd/lib/var/libkwok_engine_$V.so; [ $V = def ] && L=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$L timeout -k 10 200 python3 -u $R/tools/once_probe.py 100 $V >> $R/gpurun_out/r5b.txt 2> $R/gpurun_out/r5b.err || { tail -5 $R/gpurun_out/r5b.err; exit 4; }
done
cat $R/gpurun_out/r5b.txt
