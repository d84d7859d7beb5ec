# the C4 leg alone (tools/c4_probe.py): plain with KWOK_INGEST_PROF, then under a
# kernel trace (per-kernel stats, the timeline of the last step)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
KWOK_INGEST_PROF=1 timeout -k 10 300 python -u $R/tools/c4_probe.py --ticks 6 > $R/gpurun_out/c4_$TAG.json 2> $R/gpurun_out/c4_$TAG.err || { tail -20 $R/gpurun_out/c4_$TAG.err; exit 1; }
grep "^{" $R/gpurun_out/c4_$TAG.json
grep "kwok ingest" $R/gpurun_out/c4_$TAG.err | tail -4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4_$TAG -o run -- python3 $R/tools/c4_probe.py --ticks 2 > $R/gpurun_out/prof_c4_$TAG.log 2>&1 || exit 3
T=$(find $R/gpurun_out/prof_c4_$TAG -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 3 --out $R/gpurun_out/ktrace_c4_$TAG.txt
python3 $R/tools/timeline.py "$T" --last 45 > $R/gpurun_out/timeline_c4_$TAG.txt
cat $R/gpurun_out/timeline_c4_$TAG.txt
