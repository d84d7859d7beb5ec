#!/bin/bash
# k_emit iteration: the emitter's parity tests, then the headline bench without
# the CPU baseline (its initial_tick line carries k_emit), then a kernel trace.
# Usage: gpu_emit.sh TAG [extra pytest files]
set -o pipefail
TAG=${1:-e}
shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_emit_paths_gpu.py \
  tests/test_parity_gpu.py tests/test_custom_template_gpu.py "$@" > $R/gpurun_out/tests_$TAG.log 2>&1
trc=$?
tail -4 $R/gpurun_out/tests_$TAG.log
[ $trc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/tests_$TAG.log | head -20; exit $trc; }
timeout -k 10 300 python bench.py --cpu-baseline 0 > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err || { tail -20 $R/gpurun_out/bench_$TAG.err; exit 3; }
python3 -c "import json; d=json.load(open('$R/gpurun_out/bench_$TAG.json')); i=d['initial_tick']; c=d['churn']; print('step %.1f us  initial wall %.2f ms kernel %.2f ms k_emit %.3f ms frac %.3f  churn tick %.2f ms k_emit %.3f ms' % (d['ms_per_step']*1e3, i['wall_ms'], i['kernel_ms'], i['k_emit_ms'], i['emit_roofline']['frac'], c['tick_ms'], c['k_emit_ms']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 2 --flap-ticks 0 > $R/gpurun_out/bench_${TAG}_prof.json 2>&1 || exit 4
grep -h "k_emit\|k_tick" $R/gpurun_out/prof_$TAG/run_kernel_stats.csv
exit 0
