#!/bin/bash
# A/B of two engine builds on one box: alternating headline bench runs.
# Usage: ab_bench.sh LIB_A LIB_B [rounds]
R=$GRAFT_REPO_ROOT
for i in $(seq ${3:-3}); do
  for L in "$1" "$2"; do
    KWOK_ENGINE_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 200 --cpu-baseline 0 --churn-ticks 0 --flap-ticks 0 --roofline-ticks 20 > $R/gpurun_out/ab.json 2>/dev/null || { echo "FAIL $L"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/ab.json')); print('%-40s step %.1f us  k_tick %.1f us  frac %.3f' % (sys.argv[1], d['ms_per_step']*1e3, d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac']))" "$(basename $L)"
  done
done
