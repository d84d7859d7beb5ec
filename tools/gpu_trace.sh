#!/bin/bash
# per-block k_tick phase stamps (KWOK_TICK_TRACE=1) for floor and C2.  Usage: gpu_trace.sh TAG [HBFIRST...]
set -o pipefail
TAG=${1:-x}; shift
for HF in ${@:-0}; do
  for N in 1000 100000; do
    KWOK_TICK_TRACE=1 KWOK_TICK_HB_FIRST=$HF timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --steps 20 --roofline-ticks 5 > gpurun_out/trace_${TAG}_${HF}_${N}.json 2> gpurun_out/trace_${TAG}_${HF}_${N}.err || exit $?
    echo "== hb_first $HF nodes $N"; grep "kwok trace" gpurun_out/trace_${TAG}_${HF}_${N}.err | grep -v " - "
    KWOK_TICK_HB_FIRST=$HF timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --roofline-ticks 20 > gpurun_out/bench_${TAG}_${HF}_${N}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('ms/step %.4f kernel_us %.1f' % (d['ms_per_step'], d['phase_ms_per_tick']['kernel']*1e3))" gpurun_out/bench_${TAG}_${HF}_${N}.json
  done
done
