#!/bin/bash
# k_tick knob sweep at C2 (and floor): streamer count, chain priority.  Usage: gpu_knobs.sh TAG
set -o pipefail
TAG=${1:-x}
run() {  # name env...
  local name=$1; shift
  for N in 1000 100000; do
    env "$@" timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --roofline-ticks 20 > gpurun_out/knob_${TAG}_${name}_${N}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-14s %6s' % (sys.argv[2], sys.argv[3]), 'ms/step %.4f' % d['ms_per_step'], {k: round(v*1e3,1) for k,v in d['phase_ms_per_tick'].items() if v})" gpurun_out/knob_${TAG}_${name}_${N}.json $name $N
  done
}
run base KWOK_X=0 || exit $?
run prio KWOK_TICK_PRIO=1 || exit $?
run s128 KWOK_TICK_STREAMERS=128 || exit $?
run s512 KWOK_TICK_STREAMERS=512 || exit $?
run s128prio KWOK_TICK_STREAMERS=128 KWOK_TICK_PRIO=1 || exit $?
run s1024 KWOK_TICK_STREAMERS=1024 || exit $?
