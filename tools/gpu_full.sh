#!/bin/bash
# One GPU call for a round checkpoint: parity tests, smoke, bench (default run),
# kernel-trace profile, then the FETCH_SIZE / WRITE_SIZE PMC passes, all
# summarised under gpurun_out/.  Each GPU step has its own time limit; the script
# stops at the first failure.  Usage: gpu_full.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
# (SKIP_TESTS=1: the suite ran green on this build in an earlier call)
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 960 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/tests_$TAG.log 2>&1
  trc=$?
  tail -6 $R/gpurun_out/tests_$TAG.log
  [ $trc -eq 0 ] || { grep -E "FAILED|Error" $R/gpurun_out/tests_$TAG.log | head -20; exit $trc; }
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/smoke_$TAG.log; exit 5; }
timeout -k 10 400 python bench.py > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err || { tail -20 $R/gpurun_out/bench_$TAG.err; exit 3; }
cut -c1-900 $R/gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 50 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --c2 0 > $R/gpurun_out/bench_${TAG}_prof.json 2>&1 || exit 4
T=$(find $R/gpurun_out/prof_$TAG -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 45 --out $R/gpurun_out/ktrace_$TAG.txt || exit 6
# the heartbeat-once steady tick alone (k_once; tools/once_probe.py: queued, then blocking ticks)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_once_$TAG -o run -- python3 $R/tools/once_probe.py 100 prof > $R/gpurun_out/bench_${TAG}_once_prof.json 2>&1 || exit 8
T=$(find $R/gpurun_out/prof_once_$TAG -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 100 --out $R/gpurun_out/ktrace_once_$TAG.txt || exit 9
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_$C -o run -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --c2 0 > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1 || exit 7
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_FETCH_SIZE $R/gpurun_out/pmc_${TAG}_WRITE_SIZE $R/gpurun_out/pmc_${TAG}.json --kernels $R/kwok_amd/csrc/kernels.hip \
  --source "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace (separate passes), bench.py --steps 20 --warmup 3, 1M nodes x 10M pods, 1x MI355X"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_once_${TAG}_$C -o run -- python3 $R/tools/once_probe.py 30 pmc > $R/gpurun_out/pmc_once_${TAG}_$C.log 2>&1 || exit 10
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_once_${TAG}_FETCH_SIZE $R/gpurun_out/pmc_once_${TAG}_WRITE_SIZE $R/gpurun_out/pmc_once_${TAG}.json --kernels $R/kwok_amd/csrc/kernels.hip \
  --source "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace (separate passes), tools/once_probe.py 30 (KWOK_CFG_HEARTBEAT_ONCE steady ticks: k_once), 1M nodes x 10M pods, 1x MI355X"
# the C4 churn tick on the heartbeat-once engine: kernel trace + timeline, FETCH_SIZE / WRITE_SIZE
bash $R/tools/gpu_c4once.sh $TAG > $R/gpurun_out/c4once_${TAG}_summary.txt 2>&1 || { tail -20 $R/gpurun_out/c4once_${TAG}_summary.txt; exit 11; }
tail -8 $R/gpurun_out/c4once_${TAG}_summary.txt
exit 0
