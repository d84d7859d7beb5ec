#!/bin/bash
# Fused pod emission A/B (k_pod_jobs<true> vs k_pod_jobs + k_emit): emission
# parity tests, then the bench's initial tick and churn legs, fused and not.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_emit_paths_gpu.py tests/test_c4_churn_gpu.py tests/test_parity_gpu.py tests/test_c3_8rank_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $R/gpurun_out/r6b_t.log 2>&1
rc=$?; tail -3 $R/gpurun_out/r6b_t.log; [ $rc -eq 0 ] || exit $rc
for V in "" 0 "" 0; do
  KWOK_FUSE_EMIT=$V timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 > $R/gpurun_out/r6b_x$V.json 2> $R/gpurun_out/r6b_x$V.err || { tail -5 $R/gpurun_out/r6b_x$V.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); i=d['initial_tick']; c=d['churn']; print('fuse', sys.argv[2], 'init wall %.3f emission %.3f | churn step %.3f tick %.3f emission %.3f | steady %.4f' % (i['wall_ms'], i['emission_ms'], c['ms_per_step'], c['median_ms']['tick'], c['emission_ms'], d['ms_per_step']))" $R/gpurun_out/r6b_x$V.json "auto$V"
done
