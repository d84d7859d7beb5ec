#!/bin/bash
# The heartbeat-once leg with its queued warmup, three times.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 1 > $R/gpurun_out/ran_$i.json 2> $R/gpurun_out/ran_$i.err || exit 2
  python3 -c "import json; d=json.load(open('$R/gpurun_out/ran_$i.json')); o=d['heartbeat_once']; print('steady %.4f ms | once %.4f ms/step -> %.2f G/s, kernel %.4f' % (d['ms_per_step'], o['ms_per_step'], o['value']/1e9, o['kernel_ms']))"
done
exit 0
