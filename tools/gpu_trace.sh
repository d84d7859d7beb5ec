#!/bin/bash
# per-block k_tick phase stamps (KWOK_TICK_TRACE=1) for floor and C2.  Usage: gpu_trace.sh TAG
set -o pipefail
TAG=${1:-x}
for N in 1000 100000; do
  KWOK_TICK_TRACE=1 timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --no-queue --steps 20 --roofline-ticks 5 > gpurun_out/trace_${TAG}_${N}.json 2> gpurun_out/trace_${TAG}_${N}.err || exit $?
  echo "== nodes $N"; grep "kwok trace" gpurun_out/trace_${TAG}_${N}.err
done
