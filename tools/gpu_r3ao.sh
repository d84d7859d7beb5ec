#!/bin/bash
# Steady tick: heartbeat stream store flavour (KWOK_HB_NT) x streamers' share, env-only A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for v in "nt860:KWOK_X=0" "pl860:KWOK_HB_NT=0" "pl921:KWOK_HB_NT=0 KWOK_TICK_STREAM_SHARE=921" "pl800:KWOK_HB_NT=0 KWOK_TICK_STREAM_SHARE=800" "nt860b:KWOK_X=0" "pl860b:KWOK_HB_NT=0" "nt900:KWOK_TICK_STREAM_SHARE=900" "nt820:KWOK_TICK_STREAM_SHARE=820"; do
  n=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --steps 200 --cpu-baseline 0 --roofline-ticks 20 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/rao_$n.json 2> $R/gpurun_out/rao_$n.err || { tail -5 $R/gpurun_out/rao_$n.err; exit 2; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/rao_$n.json')); r=d['roofline']; print('%-7s step %.4f ms  k_tick %.4f ms  frac %.3f  classify %.4f' % ('$n', d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['phase_ms_per_tick']['classify']))"
done
exit 0
