#!/bin/bash
# k_emit (node inits) beside the fused k_pod_jobs: parity tests, then the
# initial tick A/B (KWOK_EMIT_CONCURRENT default vs 0), twice, one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_emit_paths_gpu.py tests/test_parity_gpu.py tests/test_c3_8rank_gpu.py tests/test_controller_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $R/gpurun_out/r6e_t.log 2>&1
rc=$?; tail -2 $R/gpurun_out/r6e_t.log; [ $rc -eq 0 ] || exit $rc
for V in "" 0 "" 0; do
  KWOK_EMIT_CONCURRENT=$V timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --churn-ticks 0 > $R/gpurun_out/r6e_x$V.json 2> $R/gpurun_out/r6e_x$V.err || { tail -5 $R/gpurun_out/r6e_x$V.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); i=d['initial_tick']; print('concurrent', sys.argv[2], 'init wall %.3f kernels %.3f emission %.3f | steady %.4f' % (i['wall_ms'], i['kernel_ms'], i['emission_ms'], d['ms_per_step']))" $R/gpurun_out/r6e_x$V.json "default$V"
done
