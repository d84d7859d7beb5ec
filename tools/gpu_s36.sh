# k_json_nodes (C5 from its node documents, 10k per batch): kernel time by
# documents per wave (64 / 32 / 16) and SQ counters at 64 (where the waves' cycles go)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for L in 64 32 16; do
  KWOK_JSON_NODE_LANES=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s36_$L -o run -- python3 $R/bench.py --leg flap_once --flap-ticks 6 > $R/gpurun_out/prof_s36_$L.log 2>&1 || exit 5
  T=$(find $R/gpurun_out/prof_s36_$L -name 'run_kernel_trace.csv' | head -n 1)
  python3 $R/tools/trace_summary.py "$T" --last 6 --out $R/gpurun_out/ktrace_s36_$L.txt
  echo "lanes $L: $(grep -E 'k_json_nodes' $R/gpurun_out/ktrace_s36_$L.txt)"
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/sq_s36_$i -o run -- python3 $R/bench.py --leg flap_once --flap-ticks 4 > $R/gpurun_out/sq_s36_$i.log 2>&1 || exit 7
done
python3 $R/tools/sq_summary.py $R/gpurun_out/sq_s36.txt $R/gpurun_out/sq_s36_1 $R/gpurun_out/sq_s36_2 --kernel k_json_nodes --title "SQ counters, k_json_nodes (C5 from node documents, 10k per batch)" || exit 9
cat $R/gpurun_out/sq_s36.txt
