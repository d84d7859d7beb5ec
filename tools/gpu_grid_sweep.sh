#!/bin/bash
# k_tick grid sweep: chain blocks per CU x streamer blocks per CU x {floor (1k nodes), C2}.  Usage: gpu_grid_sweep.sh TAG
set -o pipefail
TAG=${1:-x}
for BPC in 1 2; do
 for SPC in 1 2; do
  for N in 1000 100000; do
    KWOK_TICK_BLOCKS_PER_CU=$BPC KWOK_TICK_STREAMERS_PER_CU=$SPC timeout -k 10 300 python bench.py --nodes-per-rank $N --cpu-baseline 0 --roofline-ticks 20 > gpurun_out/sweep_${TAG}_${BPC}_${SPC}_${N}.json 2> gpurun_out/sweep_${TAG}_${BPC}_${SPC}_${N}.err || exit $?
    python - gpurun_out/sweep_${TAG}_${BPC}_${SPC}_${N}.json $BPC $SPC $N <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ph = {k: round(v * 1e3, 1) for k, v in d["phase_ms_per_tick"].items()}
print("chain/CU", sys.argv[2], "stream/CU", sys.argv[3], "nodes", sys.argv[4], "ms/step %.4f" % d["ms_per_step"], "phases_us", ph,
      "frac %.3f" % d["roofline"]["frac"])
PY
  done
 done
done
