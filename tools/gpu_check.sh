#!/bin/bash
# One GPU call during development: the -m gpu tests, then a kernel trace of the
# bench at a given size.  Each GPU step has its own time limit; stops at the first failure.
# Usage: gpu_check.sh TAG [NODES] [extra bench args...]
set -o pipefail
TAG=${1:-x}
NODES=${2:-1000000}
shift 2
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $R/gpurun_out/tests_$TAG.log 2>&1
trc=$?
tail -4 $R/gpurun_out/tests_$TAG.log
[ $trc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/tests_$TAG.log | head -20; exit $trc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --nodes-per-rank $NODES --steps 20 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 "$@" > $R/gpurun_out/prof_$TAG.json 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.json; exit 4; }
T=$(find $R/gpurun_out/prof_$TAG -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 20 --out $R/gpurun_out/ktrace_$TAG.txt
