# the bucket sort alone (tools/sort_bench.hip, built in tools/_build) against a host
# stable sort: the 8-wave scatter (1M / 777,777 / 100 records over 4096 buckets, all
# records in one bucket), the 4-wave one (8192 buckets), with a kernel trace of the first
set -o pipefail
R=$GRAFT_REPO_ROOT
B=$R/tools/_build/sort_bench_base
for a in "1000000 4096" "777777 4096" "100 4096" "5000 1" "1000000 8192" "4097 8192"; do
  timeout -k 10 60 $B $a || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sortb_s40 -o run -- $B 1000000 4096 > $R/gpurun_out/sortb_s40.log 2>&1 || exit 2
T=$(find $R/gpurun_out/sortb_s40 -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 10 | grep k_bs
