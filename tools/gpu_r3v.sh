#!/bin/bash
# Round-3 checkpoint V (final-build profile): the GPU suite, smoke, the default
# bench, the C5 node-ingest phases (spinning worker pool, per-slot refs), the
# kernel trace and the FETCH_SIZE / WRITE_SIZE PMC passes of the steady tick.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_full.sh r3v || exit $?
KWOK_INGEST_PROF=1 timeout -k 10 400 python $R/bench.py --steps 10 --churn-ticks 0 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 8 > $R/gpurun_out/r3v_flap.json 2> $R/gpurun_out/r3v_flap.err || exit 9
grep "9990 node" $R/gpurun_out/r3v_flap.err | tail -4
python3 -c "import json; f=json.load(open('$R/gpurun_out/r3v_flap.json'))['flap']; print('flap: step %.3f ingest %.3f tick %.3f' % (f['ms_per_step'], f['ingest_ms'], f['tick_ms']))"
exit 0
