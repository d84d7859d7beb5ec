#!/bin/bash
# the GPU pod codec checkpoint: its tests (tests/test_json_gpu.py), then the
# k_once / parity tests as a regression check.  Usage: gpu_json.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_json_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/json_tests_$TAG.log 2>&1
rc=$?
tail -25 $R/gpurun_out/json_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
exit 0
