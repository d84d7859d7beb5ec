# SQ counters of the C4 ingest's kernels (k_ing_apply above all: where its waves' cycles go)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/sq_s41_$i -o run -- python3 $R/tools/c4_probe.py --ticks 2 --once > $R/gpurun_out/sq_s41_$i.log 2>&1 || exit 7
done
python3 $R/tools/sq_summary.py $R/gpurun_out/sq_s41.txt $R/gpurun_out/sq_s41_1 $R/gpurun_out/sq_s41_2 --last 4 --kernel k_ing_apply --kernel k_ing_prep --kernel k_bs_scatter --title "SQ counters, the C4 ingest kernels (tools/c4_probe.py --ticks 2 --once)" || exit 9
cat $R/gpurun_out/sq_s41.txt
