#!/bin/bash
# Round-3 checkpoint A: the 8-rank C3 test, the churn leg through the
# multi-rank tick (one-rank RCCL communicator), and a default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_c3_8rank_gpu.py -x -v --timeout 1000 --timeout-method thread > $R/gpurun_out/r3a_c3.log 2>&1
rc=$?
tail -5 $R/gpurun_out/r3a_c3.log
[ $rc -eq 0 ] || exit $rc
KWOK_FORCE_MULTI=1 timeout -k 10 400 python bench.py --steps 20 --cpu-baseline 0 --flap-ticks 0 > $R/gpurun_out/r3a_multi.json 2> $R/gpurun_out/r3a_multi.err || { tail -20 $R/gpurun_out/r3a_multi.err; exit 3; }
timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/r3a_bench.json 2> $R/gpurun_out/r3a_bench.err || { tail -20 $R/gpurun_out/r3a_bench.err; exit 4; }
cut -c1-600 $R/gpurun_out/r3a_bench.json
exit 0
