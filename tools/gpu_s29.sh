# C4 with the tick behind the batch (heartbeat-once engine): the last chunk's
# results beside the tick's kernels (default), after its k_tick launch
# (KWOK_INGEST_RAT=1) or after all its kernels (2); A/B, parity under RAT=1, trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
KWOK_INGEST_RAT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingest_tick_gpu.py \
  tests/test_c4_churn_gpu.py -k "tick or together" > gpurun_out/s29_tests.txt 2>&1 || { tail -30 gpurun_out/s29_tests.txt; exit 3; }
tail -1 gpurun_out/s29_tests.txt
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh rat0=- rat1=-=KWOK_INGEST_RAT=1 rat2=-=KWOK_INGEST_RAT=2 rat0b=- rat1b=-=KWOK_INGEST_RAT=1 > /dev/null || exit 4
for v in rat0 rat1 rat2 rat0b rat1b; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
cd /tmp && export TMPDIR=/tmp
KWOK_INGEST_RAT=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/prof_s29 -o run -- python3 $R/tools/c4_probe.py --ticks 3 --together --once > $R/gpurun_out/prof_s29.log 2>&1 || exit 5
T=$(find $R/gpurun_out/prof_s29 -name 'run_kernel_trace.csv' | head -n 1)
M=$(find $R/gpurun_out/prof_s29 -name 'run_memory_copy_trace.csv' | head -n 1)
python3 $R/tools/timeline.py "$T" --last 30 --copies "$M" > $R/gpurun_out/timeline_s29.txt
cat $R/gpurun_out/timeline_s29.txt
