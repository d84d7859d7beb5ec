#!/bin/bash
# the two-rank engine test that hung in r4i, traced; then the one-rank RCCL tests
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
KWOK_TEST_TRACE=1 timeout -k 10 170 python -u -m pytest $R/tests/test_dist_gpu.py -k "inline" -x -v -s --timeout 150 --timeout-method thread > $R/gpurun_out/r4j_dist.log 2>&1
rc=$?; tail -40 $R/gpurun_out/r4j_dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 170 python -u -m pytest $R/tests/test_rccl_gpu.py -x -v --timeout 150 --timeout-method thread > $R/gpurun_out/r4j_rccl.log 2>&1
rc=$?; tail -5 $R/gpurun_out/r4j_rccl.log; exit $rc
