#!/bin/bash
# PMC passes (counters in their own runs, kernel-trace only): FETCH_SIZE, WRITE_SIZE,
# summarised per launch into gpurun_out/pmc_TAG.json.  Usage: gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_$C -o run -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1 || exit $?
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_FETCH_SIZE $R/gpurun_out/pmc_${TAG}_WRITE_SIZE $R/gpurun_out/pmc_${TAG}.json \
  --source "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace (separate passes), bench.py --steps 20 --warmup 3, C2 100k nodes x 1M pods, 1x MI355X"
