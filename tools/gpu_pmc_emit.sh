#!/bin/bash
# SQ counters of the initial tick's k_emit (one launch; no churn / flap ticks).  Usage: gpu_pmc_emit.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_FLAT SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/pmce_${TAG}_$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 > $R/gpurun_out/pmce_${TAG}_$i.log 2>&1 || exit 7
done
for i in 1 2; do python3 $R/tools/pmc_dump.py $R/gpurun_out/pmce_${TAG}_$i --kernel k_emit; done
