#!/bin/bash
# steady tick: stream share sweep on the new kernels; one-rank RCCL (FORCE_MULTI) churn leg under a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
: > $R/gpurun_out/r4g.txt
for SH in 860 800 830 890 860 800; do
  KWOK_TICK_STREAM_SHARE=$SH timeout -k 10 300 python3 $R/bench.py --steps 100 --cpu-baseline 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/r4g_b.json 2> $R/gpurun_out/r4g_b.err || { tail -5 $R/gpurun_out/r4g_b.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('share', sys.argv[2], 'steady', round(d['ms_per_step'],4), 'k_tick', round(d['roofline']['avg_launch_ms'],4), 'classify', round(d['state_only']['classify_ms'],4))" $R/gpurun_out/r4g_b.json $SH >> $R/gpurun_out/r4g.txt
done
cat $R/gpurun_out/r4g.txt
cd /tmp && export TMPDIR=/tmp
KWOK_FORCE_MULTI=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4g_multi -o run -- python3 $R/bench.py --steps 30 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --churn-ticks 3 > $R/gpurun_out/r4g_multi.json 2> $R/gpurun_out/r4g_multi.err || { tail -5 $R/gpurun_out/r4g_multi.err; exit 5; }
python3 - <<'PY'
import json
d=json.load(open('/root/repo/gpurun_out/r4g_multi.json'))
print('multi steady', d['ms_per_step'], 'k_tick', d['roofline']['avg_launch_ms'], 'phases', {k: round(v,4) for k,v in d['phase_ms_per_tick'].items()})
for k in ('churn','churn_events'):
    c=d[k]; print(k, round(c['ms_per_step'],3), 'ingest', round(c['ingest_ms'],3), 'tick', round(c['tick_ms'],3), 'kernel', round(c['kernel_ms'],3), 'xch', c['exchange_ms'])
PY
