#!/bin/bash
# Chunked pod ingest with the batch copied to HBM by the copy engine (KWOK_INGEST_ZC=0)
# against reading it in place, over the chunk size.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for zc in 0 1; do
for ch in 100000000 524288 262144; do
  KWOK_INGEST_ZC=$zc KWOK_INGEST_CHUNK=$ch KWOK_INGEST_PROF=1 timeout -k 10 300 python bench.py --steps 10 --churn-ticks 6 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 0 > $R/gpurun_out/rae_churn${zc}_$ch.json 2> $R/gpurun_out/rae_churn${zc}_$ch.err || exit 2
  python3 -c "import json; c=json.load(open('$R/gpurun_out/rae_churn${zc}_$ch.json'))['churn']; print('zc $zc chunk $ch: step %.3f (median %.3f) ingest %.3f (median %.3f) tick %.3f' % (c['ms_per_step'], c['median_ms']['step'], c['ingest_ms'], c['median_ms']['ingest'], c['tick_ms']))"
  grep "kwok ingest" $R/gpurun_out/rae_churn${zc}_$ch.err | tail -5
done
done
exit 0
