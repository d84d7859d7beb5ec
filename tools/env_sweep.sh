#!/bin/bash
# k_tick launch-shape sweep at 1M nodes x 10M pods: one bench run per setting
# (diagnostic env knobs of engine.cpp), ms/step and the k_tick event time.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
run() {
  env "$@" timeout -k 10 120 python3 $R/bench.py --steps 100 --warmup 3 --cpu-baseline 0 --roofline-ticks 20 --churn-ticks 0 --flap-ticks 0 > $R/gpurun_out/sweep.json 2>/dev/null || { echo "FAIL $*"; return 1; }
  python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/sweep.json')); p=d['phase_ms_per_tick']; print('%-60s step %.1f us  k_tick %.1f us  classify %.1f stream %.1f' % (sys.argv[1], d['ms_per_step']*1e3, p['kernel']*1e3, p['classify']*1e3, p['stream']*1e3))" "$*"
}
run X=0
run KWOK_TICK_NO_STREAM=1
run KWOK_TICK_STREAM_SHARE=1024
run KWOK_TICK_STREAMERS_PER_CU=2
run KWOK_TICK_STREAMERS_PER_CU=2 KWOK_TICK_STREAM_SHARE=1024
run KWOK_TICK_BLOCKS_PER_CU=2
run KWOK_TICK_BLOCKS_PER_CU=2 KWOK_TICK_STREAM_SHARE=1024
run KWOK_TICK_PRIO=1
run KWOK_TICK_STREAM_SHARE=960
run KWOK_TICK_STREAM_SHARE=880
run KWOK_TICK_STREAMERS_PER_CU=2 KWOK_TICK_STREAM_SHARE=960
