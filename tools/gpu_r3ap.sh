#!/bin/bash
# Chain blocks per CU (KWOK_TICK_BLOCKS_PER_CU) on the steady and the churn tick, env-only A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for v in "c1:KWOK_X=0" "c2:KWOK_TICK_BLOCKS_PER_CU=2" "c1b:KWOK_X=0" "c2b:KWOK_TICK_BLOCKS_PER_CU=2"; do
  n=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --steps 100 --cpu-baseline 0 --roofline-ticks 20 --churn-ticks 4 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/rap_$n.json 2> $R/gpurun_out/rap_$n.err || { tail -5 $R/gpurun_out/rap_$n.err; exit 2; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/rap_$n.json')); c=d['churn']; i=d['initial_tick']; print('%-4s steady %.4f ms | churn tick %.3f kernels %.3f k_emit %.3f | initial %.3f' % ('$n', d['ms_per_step'], c['tick_ms'], c['kernel_ms'], c['k_emit_ms'], i['wall_ms']))"
done
exit 0
