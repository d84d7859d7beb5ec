# C4 with the tick behind the batch (heartbeat-once engine): the creates' handles
# written into the caller's page-locked array by the kernel (default) or into HBM
# and copied back (KWOK_INGEST_NEW_MAPPED=0) - the kernel's host writes beside
# the tick's persistent blocks - A/B twice, then the kernel trace of the copy form
set -o pipefail
R=$GRAFT_REPO_ROOT
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh nm1=- nm0=-=KWOK_INGEST_NEW_MAPPED=0 nm1b=- nm0b=-=KWOK_INGEST_NEW_MAPPED=0 > /dev/null || exit 4
for v in nm1 nm0 nm1b nm0b; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
cd /tmp && export TMPDIR=/tmp
KWOK_INGEST_NEW_MAPPED=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/prof_s27 -o run -- python3 $R/tools/c4_probe.py --ticks 3 --together --once > $R/gpurun_out/prof_s27.log 2>&1 || exit 5
T=$(find $R/gpurun_out/prof_s27 -name 'run_kernel_trace.csv' | head -n 1)
M=$(find $R/gpurun_out/prof_s27 -name 'run_memory_copy_trace.csv' | head -n 1)
python3 $R/tools/timeline.py "$T" --last 30 --copies "$M" > $R/gpurun_out/timeline_s27.txt
cat $R/gpurun_out/timeline_s27.txt
