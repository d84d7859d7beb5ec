#!/bin/bash
# Quick GPU check: the GPU test files given (default: all), then bench without
# the CPU baseline.  Usage: gpu_quick.sh TAG [pytest selectors...]
set -o pipefail
TAG=${1:-x}
shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -x -v -m gpu --timeout 600 --timeout-method thread --durations=8 > $R/gpurun_out/tests_$TAG.log 2>&1
trc=$?
tail -14 $R/gpurun_out/tests_$TAG.log
[ $trc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/tests_$TAG.log | head -30; exit $trc; }
timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err || { tail -20 $R/gpurun_out/bench_$TAG.err; exit 3; }
cut -c1-600 $R/gpurun_out/bench_$TAG.json
python3 -c "import json;d=json.load(open('$R/gpurun_out/bench_$TAG.json'));print(json.dumps(d.get('churn'),indent=0))"
