#!/bin/bash
# A checkpoint without profile passes (kernels.hip unchanged since the stored
# PMC summaries): the whole GPU suite, smoke, and the default bench run.
# Usage: gpu_final.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 960 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/tests_$TAG.log 2>&1
trc=$?
tail -4 $R/gpurun_out/tests_$TAG.log
[ $trc -eq 0 ] || { grep -E "FAILED|Error" $R/gpurun_out/tests_$TAG.log | head -20; exit $trc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/smoke_$TAG.log; exit 5; }
timeout -k 10 400 python bench.py > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err || { tail -20 $R/gpurun_out/bench_$TAG.err; exit 3; }
cut -c1-600 $R/gpurun_out/bench_$TAG.json
