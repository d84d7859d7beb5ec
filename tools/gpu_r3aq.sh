#!/bin/bash
# Final tree: smoke + the default bench line (as the driver runs them).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/raq_smoke.log 2>&1 || { tail -20 $R/gpurun_out/raq_smoke.log; exit 5; }
tail -1 $R/gpurun_out/raq_smoke.log
timeout -k 10 400 python bench.py > $R/gpurun_out/raq_bench.json 2> $R/gpurun_out/raq_bench.err || { tail -20 $R/gpurun_out/raq_bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$R/gpurun_out/raq_bench.json')); c=d['churn']; f=d['flap']; o=d['heartbeat_once']; print('step %.4f (%.2f G/s, frac %.3f, traffic %s) | churn %.3f | flap %.3f | once %.4f | initial %.3f' % (d['ms_per_step'], d['value']/1e9, d['roofline']['frac'], d['roofline']['traffic'], c['ms_per_step'], f['ms_per_step'], o['ms_per_step'], d['initial_tick']['wall_ms']))"
exit 0
