#!/bin/bash
# host completion wait: blocking stream sync vs spinning on an event.  Usage: gpu_sync.sh TAG
set -o pipefail
TAG=${1:-x}
for SY in block spin; do
  for N in 1000 100000; do
    KWOK_SYNC=$SY timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --roofline-ticks 20 > gpurun_out/sync_${TAG}_${SY}_${N}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], 'ms/step %.4f kernel_us %.1f host_us' % (d['ms_per_step'], d['phase_ms_per_tick']['kernel']*1e3), {k: round(v*1e3,1) for k,v in d['host_ms_per_tick'].items()})" gpurun_out/sync_${TAG}_${SY}_${N}.json $SY $N
  done
done
