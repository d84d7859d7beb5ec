#!/bin/bash
# steady-tick A/B against the round-3 kernels (lib/var/..._orig); churn steps with per-chunk ingest times
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
: > $R/gpurun_out/r4l.txt
for V in def nf0 np1 def nf0 np1; do
  L=$R/kwok_amd/lib/var/libkwok_engine_$V.so; [ $V = def ] && L=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 100 --cpu-baseline 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 > $R/gpurun_out/r4l_b.json 2> $R/gpurun_out/r4l_b.err || { tail -5 $R/gpurun_out/r4l_b.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'steady', round(d['ms_per_step'],4), 'k_tick', round(d['roofline']['avg_launch_ms'],4), 'classify', round(d['state_only']['classify_ms'],4))" $R/gpurun_out/r4l_b.json $V | tee -a $R/gpurun_out/r4l.txt
done
KWOK_INGEST_PROF=1 timeout -k 10 300 python3 $R/bench.py --steps 5 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --churn-ticks 8 > $R/gpurun_out/r4l_churn.json 2> $R/gpurun_out/r4l_churn.err || { tail -5 $R/gpurun_out/r4l_churn.err; exit 5; }
python3 -c "import json; d=json.load(open('$R/gpurun_out/r4l_churn.json')); c=d['churn']; print('churn', c['ms_per_step'], c['median_ms'], c['steps_ms'])" | tee -a $R/gpurun_out/r4l.txt
grep -E "kwok ingest|chunk" $R/gpurun_out/r4l_churn.err | tail -40
