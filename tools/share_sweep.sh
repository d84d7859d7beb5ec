#!/bin/bash
# heartbeat stream share sweep (streamers' /1024) at 1M x 10M with the non-temporal stream
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
run() {
  env "$@" timeout -k 10 120 python3 $R/bench.py --steps 200 --warmup 3 --cpu-baseline 0 --roofline-ticks 20 --churn-ticks 0 --flap-ticks 0 > $R/gpurun_out/sweep.json 2> $R/gpurun_out/sweep.err || { echo "FAIL $*"; tail -3 $R/gpurun_out/sweep.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/sweep.json')); p=d['phase_ms_per_tick']; print('%-50s step %.1f us  k_tick %.1f us  classify %.1f stream %.1f' % (sys.argv[1], d['ms_per_step']*1e3, p['kernel']*1e3, p['classify']*1e3, p['stream']*1e3))" "$*"
}
for s in 921 860 800 740 680 921; do run KWOK_TICK_STREAM_SHARE=$s; done
run KWOK_TICK_STREAMERS_PER_CU=2
run KWOK_TICK_STREAMERS_PER_CU=2 KWOK_TICK_STREAM_SHARE=800
