#!/bin/bash
# The C4 churn tick on the heartbeat-once engine (the drop-in's): c4_probe.py --once
# plain, then under a kernel trace (per-kernel stats + the timeline of the last
# steps), then FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) summarised per
# kernel.  Usage: gpu_c4once.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u $R/tools/c4_probe.py --once --ticks 6 > $R/gpurun_out/c4once_$TAG.json 2> $R/gpurun_out/c4once_$TAG.err || { tail -20 $R/gpurun_out/c4once_$TAG.err; exit 1; }
grep "^{" $R/gpurun_out/c4once_$TAG.json | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4once_$TAG -o run -- python3 $R/tools/c4_probe.py --once --ticks 4 > $R/gpurun_out/prof_c4once_$TAG.log 2>&1 || exit 3
T=$(find $R/gpurun_out/prof_c4once_$TAG -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 60 --out $R/gpurun_out/ktrace_c4once_$TAG.txt || exit 4
python3 $R/tools/timeline.py "$T" --last 60 > $R/gpurun_out/timeline_c4once_$TAG.txt || exit 4
cat $R/gpurun_out/ktrace_c4once_$TAG.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_c4once_${TAG}_$C -o run -- python3 $R/tools/c4_probe.py --once --ticks 4 > $R/gpurun_out/pmc_c4once_${TAG}_$C.log 2>&1 || exit 5
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_c4once_${TAG}_FETCH_SIZE $R/gpurun_out/pmc_c4once_${TAG}_WRITE_SIZE $R/gpurun_out/pmc_c4once_${TAG}.json --last 4 --kernels $R/kwok_amd/csrc/kernels.hip \
  --source "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace (separate passes), tools/c4_probe.py --once --ticks 4 (C4 churn ticks on the KWOK_CFG_HEARTBEAT_ONCE engine), 1M nodes x 10M pods, 1x MI355X; the last 4 launches of each kernel are churn ticks"
exit 0
