#!/bin/bash
# HBM traffic of the initial tick's emission, unfused (KWOK_FUSE_EMIT=0), beside
# the fused figures of profiles/r6c_pmc.json: FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export KWOK_FUSE_EMIT=0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_r6h_$C -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 > $R/gpurun_out/pmc_r6h_$C.log 2>&1 || exit 7
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_r6h_FETCH_SIZE $R/gpurun_out/pmc_r6h_WRITE_SIZE $R/gpurun_out/pmc_r6h.json --kernels $R/kwok_amd/csrc/kernels.hip \
  --source "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace (separate passes), KWOK_FUSE_EMIT=0, bench.py --steps 5 --warmup 2, 1M nodes x 10M pods, 1x MI355X" || exit 8
