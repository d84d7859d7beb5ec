#!/bin/bash
# heartbeat stream share (streamers vs chain blocks) sweep.  Usage: gpu_share.sh TAG
set -o pipefail
TAG=${1:-x}
for SH in ${SHARES:-1024 980 940 921 880}; do
  for N in ${NODES:-100000}; do
    KWOK_TICK_STREAM_SHARE=$SH timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --roofline-ticks 20 > gpurun_out/share_${TAG}_${SH}_${N}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('share', sys.argv[2], 'nodes', sys.argv[3], 'ms/step %.4f' % d['ms_per_step'], {k: round(v*1e3,1) for k,v in d['phase_ms_per_tick'].items() if v})" gpurun_out/share_${TAG}_${SH}_${N}.json $SH $N
  done
done
