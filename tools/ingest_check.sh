#!/bin/bash
# Ingest change check: the GPU tests that drive kwok_ingest_pods (threaded and
# serial paths, growth, churn at full size), then the churn leg with the
# ingest phase timings (KWOK_INGEST_PROF=1).  Usage: ingest_check.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_c4_churn_gpu.py tests/test_growth_gpu.py tests/test_scale_gpu.py tests/test_parity_gpu.py tests/test_cni_gpu.py > $R/gpurun_out/ingtests_$TAG.log 2>&1
rc=$?; tail -4 $R/gpurun_out/ingtests_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $R/gpurun_out/ingtests_$TAG.log | head; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --roofline-ticks 0 --flap-ticks 0 --churn-ticks 5 > $R/gpurun_out/ing_$TAG.json 2> $R/gpurun_out/ing_$TAG.err || exit 3
grep -h "kwok ingest" $R/gpurun_out/ing_$TAG.err | tail -5
