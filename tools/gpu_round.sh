#!/bin/bash
# GPU call: parity tests then bench (+ optional kernel trace).  Usage: gpu_round.sh TAG [prof]
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
trc=$?
tail -15 gpurun_out/tests_$TAG.log
[ $trc -eq 0 ] || [ $trc -eq 1 ] || exit $trc
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 3; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python bench.py --nodes-per-rank 1000 --cpu-baseline 0 --roofline-ticks 10 > gpurun_out/bench_${TAG}_floor.json 2>/dev/null && cut -c1-400 gpurun_out/bench_${TAG}_floor.json
if [ "$2" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 50 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 > $R/gpurun_out/bench_${TAG}_prof.json 2>&1 || exit 4
fi
exit $trc
