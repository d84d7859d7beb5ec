#!/bin/bash
# streamer start delay sweep at C2.  Usage: gpu_delay.sh TAG
set -o pipefail
TAG=${1:-x}
for D in 0 2000 4000 6000 8000; do
  for SPC in 1 2; do
    KWOK_TICK_STREAM_DELAY_NS=$D KWOK_TICK_STREAMERS_PER_CU=$SPC timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline-ticks 20 > gpurun_out/delay_${TAG}_${D}_${SPC}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('delay_ns', sys.argv[2], 'spc', sys.argv[3], 'ms/step %.4f' % d['ms_per_step'], {k: round(v*1e3,1) for k,v in d['phase_ms_per_tick'].items() if v})" gpurun_out/delay_${TAG}_${D}_${SPC}.json $D $SPC
  done
done
