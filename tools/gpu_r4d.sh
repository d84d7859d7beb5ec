#!/bin/bash
# k_tick row batching A/B: heartbeat-once probe per variant, a trace of rb3, steady + churn bench orig vs rb3
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
: > $R/gpurun_out/r4d.txt
for V in orig rb2 rb3 rb4 orig rb3; do
  KWOK_ENGINE_LIB=$R/kwok_amd/lib/var/libkwok_engine_$V.so timeout -k 10 120 python3 $R/tools/once_probe.py 100 $V >> $R/gpurun_out/r4d.txt 2> $R/gpurun_out/r4d_$V.err || { tail -5 $R/gpurun_out/r4d_$V.err; exit 2; }
done
KWOK_ENGINE_LIB=$R/kwok_amd/lib/var/libkwok_engine_rb3.so KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=8 timeout -k 10 120 python3 $R/tools/once_probe.py 50 trace-rb3 >> $R/gpurun_out/r4d.txt 2> $R/gpurun_out/r4d_trace.err || { tail -5 $R/gpurun_out/r4d_trace.err; exit 3; }
grep "kwok trace" $R/gpurun_out/r4d_trace.err >> $R/gpurun_out/r4d.txt
for V in orig rb3; do
  KWOK_ENGINE_LIB=$R/kwok_amd/lib/var/libkwok_engine_$V.so timeout -k 10 300 python3 $R/bench.py --steps 50 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r4d_bench_$V.json 2> $R/gpurun_out/r4d_bench_$V.err || { tail -5 $R/gpurun_out/r4d_bench_$V.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['churn']; print(sys.argv[2], 'steady', round(d['ms_per_step'],4), 'k_tick', round(d['roofline']['avg_launch_ms'],4), 'classify', round(d['state_only']['classify_ms'],4), 'churn', round(c['ms_per_step'],3), 'tick', round(c['tick_ms'],3), 'kern', round(c['kernel_ms'],3), 'init', round(d['initial_tick']['wall_ms'],3))" $R/gpurun_out/r4d_bench_$V.json $V >> $R/gpurun_out/r4d.txt
done
cat $R/gpurun_out/r4d.txt
