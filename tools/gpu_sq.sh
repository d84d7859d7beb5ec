#!/bin/bash
# SQ counters (where the waves' cycles go, instructions per wave, store width) of the
# emission (k_pod_jobs<true>, the initial tick), the steady k_tick and k_once, each
# counter set in a pass of its own (8 SQ counters at most per pass).  Usage: gpu_sq.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/sq_${TAG}_$i -o run -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --c2 0 > $R/gpurun_out/sq_${TAG}_$i.log 2>&1 || exit 7
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/sq_once_${TAG}_$i -o run -- python3 $R/tools/once_probe.py 30 sq > $R/gpurun_out/sq_once_${TAG}_$i.log 2>&1 || exit 8
done
python3 $R/tools/sq_summary.py $R/gpurun_out/sq_${TAG}.txt $R/gpurun_out/sq_${TAG}_1 $R/gpurun_out/sq_${TAG}_2 --pmc $R/profiles/${PMC:-r9k_pmc.json} \
  --kernel k_pod_jobs --kernel k_tick --title "SQ counters, bench.py --steps 20 (1M x 10M, 1x MI355X): the initial tick's emission and the steady k_tick" || exit 9
python3 $R/tools/sq_summary.py $R/gpurun_out/sq_once_${TAG}.txt $R/gpurun_out/sq_once_${TAG}_1 $R/gpurun_out/sq_once_${TAG}_2 --pmc $R/profiles/${PMC_ONCE:-r9k_once_pmc.json} \
  --kernel k_once --title "SQ counters, tools/once_probe.py 30 (heartbeat-once steady ticks, 1M x 10M, 1x MI355X)" || exit 10
exit 0
