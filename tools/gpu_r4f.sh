#!/bin/bash
# once-tick variants (prefetch / batch), trace, and steady-tick A/B against the round-3 kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
: > $R/gpurun_out/r4f.txt
for V in def pf3 nopf3 orig def orig; do
  L=$R/kwok_amd/lib/var/libkwok_engine_$V.so; [ $V = def ] && L=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$L timeout -k 10 120 python3 $R/tools/once_probe.py 100 $V >> $R/gpurun_out/r4f.txt 2> $R/gpurun_out/r4f_p.err || { tail -5 $R/gpurun_out/r4f_p.err; exit 2; }
done
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=8 timeout -k 10 120 python3 $R/tools/once_probe.py 50 trace-def >> $R/gpurun_out/r4f.txt 2> $R/gpurun_out/r4f_trace.err || { tail -5 $R/gpurun_out/r4f_trace.err; exit 3; }
grep "kwok trace" $R/gpurun_out/r4f_trace.err >> $R/gpurun_out/r4f.txt
for V in def orig def orig; do
  L=$R/kwok_amd/lib/var/libkwok_engine_$V.so; [ $V = def ] && L=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 100 --cpu-baseline 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r4f_b.json 2> $R/gpurun_out/r4f_b.err || { tail -5 $R/gpurun_out/r4f_b.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'steady', round(d['ms_per_step'],4), 'k_tick', round(d['roofline']['avg_launch_ms'],4), 'classify', round(d['state_only']['classify_ms'],4), 'init', round(d['initial_tick']['wall_ms'],3))" $R/gpurun_out/r4f_b.json $V >> $R/gpurun_out/r4f.txt
done
cat $R/gpurun_out/r4f.txt
