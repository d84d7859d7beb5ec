#!/bin/bash
# C4 on the heartbeat-once engine, diagnostics: per-block phase stamps of the churn
# ticks (KWOK_TICK_TRACE), the same run fused (KWOK_FUSE_EMIT=1), and the k_pod_jobs
# per-wave timeline of the last churn tick (KWOK_JOBS_TRACE).  Usage: gpu_c4diag.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
mkdir -p $R/gpurun_out
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=3 timeout -k 10 300 python -u $R/tools/c4_probe.py --once --ticks 4 > $R/gpurun_out/c4d_trace_$TAG.json 2> $R/gpurun_out/c4d_trace_$TAG.err || { tail -20 $R/gpurun_out/c4d_trace_$TAG.err; exit 1; }
grep "kwok trace" $R/gpurun_out/c4d_trace_$TAG.err
for F in 0 1; do
  KWOK_FUSE_EMIT=$F timeout -k 10 300 python -u $R/tools/c4_probe.py --once --ticks 6 > $R/gpurun_out/c4d_fuse${F}_$TAG.json 2> $R/gpurun_out/c4d_fuse${F}_$TAG.err || { tail -20 $R/gpurun_out/c4d_fuse${F}_$TAG.err; exit 2; }
  echo "fuse=$F $(grep '^{' $R/gpurun_out/c4d_fuse${F}_$TAG.json | cut -c1-420)"
done
KWOK_JOBS_TRACE=$R/gpurun_out/c4d_jt_$TAG.bin timeout -k 10 300 python -u $R/tools/c4_probe.py --once --ticks 2 > $R/gpurun_out/c4d_jt_$TAG.json 2> $R/gpurun_out/c4d_jt_$TAG.err || { tail -20 $R/gpurun_out/c4d_jt_$TAG.err; exit 3; }
python3 $R/tools/jobs_trace.py $R/gpurun_out/c4d_jt_$TAG.bin > $R/gpurun_out/c4d_jt_$TAG.txt
head -40 $R/gpurun_out/c4d_jt_$TAG.txt
