#!/bin/bash
# Heartbeat-once leg under a kernel trace: the gap between queued k_tick launches.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ral_prof -o run -- python3 $R/bench.py --steps 50 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 1 > $R/gpurun_out/ral.json 2> $R/gpurun_out/ral.err || exit 2
python3 - <<'PY'
import csv, json
rows = list(csv.DictReader(open('/root/repo/gpurun_out/ral_prof/run_kernel_trace.csv')))
k = sorted([(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:24], r['Grid_Size_X']) for r in rows if 'k_tick' in r['Kernel_Name']])
last = k[-90:]
durs = [(e - s) / 1e3 for s, e, _, _ in last]
gaps = [(last[i + 1][0] - last[i][1]) / 1e3 for i in range(len(last) - 1)]
print('last 90 k_tick: grid', set(x[3] for x in last))
print('dur us: min %.1f med %.1f max %.1f' % (min(durs), sorted(durs)[len(durs) // 2], max(durs)))
print('gap us: min %.1f med %.1f max %.1f' % (min(gaps), sorted(gaps)[len(gaps) // 2], max(gaps)))
print('gaps', ' '.join('%.0f' % g for g in gaps[-40:]))
d = json.load(open('/root/repo/gpurun_out/ral.json')); print(d['heartbeat_once']['ms_per_step'], d['heartbeat_once']['kernel_ms'])
PY
exit 0
