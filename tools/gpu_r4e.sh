#!/bin/bash
# full GPU suite on the new kernels (podIP state bits, row batches, packed ingest), once probe A/B, default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 1000 python -u -m pytest ${TESTS:-$R/tests} -m gpu -x -v --timeout 600 --timeout-method thread > $R/gpurun_out/r4e_tests.log 2>&1
rc=$?; tail -4 $R/gpurun_out/r4e_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/r4e_tests.log | head -30; exit $rc; }
: > $R/gpurun_out/r4e.txt
timeout -k 10 120 python3 $R/tools/once_probe.py 100 rb3 >> $R/gpurun_out/r4e.txt 2> $R/gpurun_out/r4e_p.err || { tail -5 $R/gpurun_out/r4e_p.err; exit 2; }
for V in rb2 rb4 orig; do
  KWOK_ENGINE_LIB=$R/kwok_amd/lib/var/libkwok_engine_$V.so timeout -k 10 120 python3 $R/tools/once_probe.py 100 $V >> $R/gpurun_out/r4e.txt 2> $R/gpurun_out/r4e_p.err || { tail -5 $R/gpurun_out/r4e_p.err; exit 2; }
done
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=8 timeout -k 10 120 python3 $R/tools/once_probe.py 50 trace-rb3 >> $R/gpurun_out/r4e.txt 2> $R/gpurun_out/r4e_trace.err || { tail -5 $R/gpurun_out/r4e_trace.err; exit 3; }
grep "kwok trace" $R/gpurun_out/r4e_trace.err >> $R/gpurun_out/r4e.txt
cat $R/gpurun_out/r4e.txt
timeout -k 10 400 python3 $R/bench.py > $R/gpurun_out/r4e_bench.json 2> $R/gpurun_out/r4e_bench.err || { tail -20 $R/gpurun_out/r4e_bench.err; exit 4; }
python3 - <<'PY'
import json
d=json.load(open('/root/repo/gpurun_out/r4e_bench.json'))
print('steady', d['ms_per_step'], 'k_tick', d['roofline']['avg_launch_ms'], 'frac', d['roofline']['frac'], 'classify', d['state_only']['classify_ms'])
for k in ('churn','churn_events'):
    c=d[k]; print(k, round(c['ms_per_step'],3), 'ingest', round(c['ingest_ms'],3), 'tick', round(c['tick_ms'],3), 'median', {a:round(b,3) for a,b in c['median_ms'].items()})
print('flap', d['flap']['ms_per_step'], 'once', d['heartbeat_once']['ms_per_step'], d['heartbeat_once']['kernel_ms'], 'init', d['initial_tick']['wall_ms'], d['initial_tick']['k_emit_ms'])
print('cpu', d['cpu_baseline']['value'])
PY
