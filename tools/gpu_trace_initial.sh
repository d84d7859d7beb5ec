#!/bin/bash
# per-block stamps of the C2 initial tick (the bulk dirty tick).  Usage: gpu_trace_initial.sh TAG
set -o pipefail
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=0 KWOK_TICK_TRACE_COUNT=1 timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 1 --warmup 1 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 > gpurun_out/trace_init_$1.json 2> gpurun_out/trace_init_$1.err || exit $?
grep "kwok trace" gpurun_out/trace_init_$1.err
