# the C4 step's timeline with 1M-record chunks and with 512k-record chunks (the
# tick behind the batch, heartbeat-once engine): where smaller chunks lose
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in 1048576 524288; do
  KWOK_INGEST_CHUNK=$c timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/prof_s25_$c -o run -- python3 $R/tools/c4_probe.py --ticks 3 --together --once > $R/gpurun_out/prof_s25_$c.log 2>&1 || exit 5
  T=$(find $R/gpurun_out/prof_s25_$c -name 'run_kernel_trace.csv' | head -n 1)
  M=$(find $R/gpurun_out/prof_s25_$c -name 'run_memory_copy_trace.csv' | head -n 1)
  head -1 "$M"
  python3 $R/tools/timeline.py "$T" --last 40 --copies "$M" > $R/gpurun_out/timeline_s25_$c.txt
  grep '^{' $R/gpurun_out/prof_s25_$c.log | cut -c1-200
done
ls $R/gpurun_out/prof_s25_524288/*/ 2>/dev/null | head
