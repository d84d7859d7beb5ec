#!/bin/bash
# Verification of the final build: the GPU suite, smoke, the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 960 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/tests_r6d.log 2>&1
rc=$?; tail -3 $R/gpurun_out/tests_r6d.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $R/gpurun_out/tests_r6d.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke_r6d.log 2>&1 || { tail -20 $R/gpurun_out/smoke_r6d.log; exit 5; }
timeout -k 10 400 python bench.py > $R/gpurun_out/bench_r6d.json 2> $R/gpurun_out/bench_r6d.err || { tail -20 $R/gpurun_out/bench_r6d.err; exit 3; }
python3 -c "import json; d=json.load(open('$R/gpurun_out/bench_r6d.json')); c=d['churn']; i=d['initial_tick']; print('steady %.4f frac %.3f traffic %s | churn %.3f %s | flap %.3f | once %.4f | init %.3f em %.3f' % (d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], c['ms_per_step'], {k: round(v, 3) for k, v in c['median_ms'].items()}, d['flap']['ms_per_step'], d['heartbeat_once']['ms_per_step'], i['wall_ms'], i['emission_ms']))"
