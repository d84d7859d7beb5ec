#!/bin/bash
# per-block stamps of steady C2 ticks, with and without the heartbeat bodies.  Usage: gpu_trace2.sh TAG
set -o pipefail
for NS in 0 1; do
  KWOK_TICK_NO_STREAM=$NS KWOK_TICK_TRACE=1 timeout -k 10 120 python bench.py --cpu-baseline 0 --no-queue --steps 20 --roofline-ticks 5 > gpurun_out/tr2_$1_$NS.json 2> gpurun_out/tr2_$1_$NS.err || exit $?
  echo "== no_stream=$NS"; grep "kwok trace" gpurun_out/tr2_$1_$NS.err
done
