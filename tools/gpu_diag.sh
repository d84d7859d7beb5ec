#!/bin/bash
# GPU round: parity tests, then bench + per-block trace + grid sweep.  Usage: gpu_diag.sh TAG
set -o pipefail
TAG=${1:-x}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
trc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/tests_$TAG.log | tail -20
[ $trc -eq 0 ] || exit $trc
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 3; }
cut -c1-1500 gpurun_out/bench_$TAG.json
bash tools/gpu_trace.sh $TAG || exit $?
[ "$2" = "sweep" ] && { bash tools/gpu_grid_sweep.sh $TAG || exit $?; }
exit 0
