#!/bin/bash
# Round-4 final checkpoint (tools/gpu_full.sh) plus the fused-emission A/B legs
# (default rule vs KWOK_FUSE_EMIT=0) on the same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_full.sh r6c || exit $?
cd $R
for V in "" 0; do
  KWOK_FUSE_EMIT=$V timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 > $R/gpurun_out/r6c_ab$V.json 2> $R/gpurun_out/r6c_ab$V.err || { tail -5 $R/gpurun_out/r6c_ab$V.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); i=d['initial_tick']; c=d['churn']; print('fuse', sys.argv[2], 'init wall %.3f emission %.3f | churn step %.3f tick %.3f emission %.3f | steady %.4f' % (i['wall_ms'], i['emission_ms'], c['ms_per_step'], c['median_ms']['tick'], c['emission_ms'], d['ms_per_step']))" $R/gpurun_out/r6c_ab$V.json "auto$V"
done
