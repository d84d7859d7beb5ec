# the bucket sort alone (tools/sort_bench.hip) and two timing variants, each
# under a kernel trace: per-kernel means
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for V in base NO_STORE; do
  B=$R/tools/_build/sort_bench_$V
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sortb_$V -o run -- $B > $R/gpurun_out/sortb_$V.log 2>&1 || { tail -5 $R/gpurun_out/sortb_$V.log; exit 1; }
  grep mismatches $R/gpurun_out/sortb_$V.log
  T=$(find $R/gpurun_out/sortb_$V -name 'run_kernel_trace.csv' | head -n 1)
  python3 $R/tools/trace_summary.py "$T" --last 10 | grep k_bs
done
