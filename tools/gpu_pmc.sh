#!/bin/bash
# The FETCH_SIZE / WRITE_SIZE PMC passes of tools/gpu_full.sh alone (main bench leg
# and the heartbeat-once leg), for a kernels.hip change that needs its traffic
# summary refreshed (bench.py reads it only when its sha256 matches).  Usage: gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_$C -o run -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --c2 0 > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1 || exit 7
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_FETCH_SIZE $R/gpurun_out/pmc_${TAG}_WRITE_SIZE $R/gpurun_out/pmc_${TAG}.json --kernels $R/kwok_amd/csrc/kernels.hip \
  --source "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace (separate passes), bench.py --steps 20 --warmup 3, 1M nodes x 10M pods, 1x MI355X" || exit 8
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_once_${TAG}_$C -o run -- python3 $R/tools/once_probe.py 30 pmc > $R/gpurun_out/pmc_once_${TAG}_$C.log 2>&1 || exit 10
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_once_${TAG}_FETCH_SIZE $R/gpurun_out/pmc_once_${TAG}_WRITE_SIZE $R/gpurun_out/pmc_once_${TAG}.json --kernels $R/kwok_amd/csrc/kernels.hip \
  --source "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace (separate passes), tools/once_probe.py 30 (KWOK_CFG_HEARTBEAT_ONCE steady ticks: k_once), 1M nodes x 10M pods, 1x MI355X" || exit 11
exit 0
