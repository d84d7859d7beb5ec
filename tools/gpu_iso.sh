#!/bin/bash
# chain alone (no heartbeat bodies) vs full tick, C2 and floor.  Usage: gpu_iso.sh TAG
set -o pipefail
TAG=${1:-x}
for NS in 0 1; do
  for N in 1000 100000; do
    KWOK_TICK_NO_STREAM=$NS timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --roofline-ticks 20 > gpurun_out/iso_${TAG}_${NS}_${N}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('nostream', sys.argv[2], 'nodes', sys.argv[3], 'ms/step %.4f' % d['ms_per_step'], {k: round(v*1e3,1) for k,v in d['phase_ms_per_tick'].items() if v})" gpurun_out/iso_${TAG}_${NS}_${N}.json $NS $N
  done
done
