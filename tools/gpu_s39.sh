# the batch's page-locked buffers from hipHostMalloc (KWOK_HOST_ALLOC=hip) against
# mmap + hipHostRegister (default): which engine the result copies take, and C4
# (the tick behind the batch, heartbeat-once engine)
set -o pipefail
R=$GRAFT_REPO_ROOT
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh reg=- hip=-=KWOK_HOST_ALLOC=hip reg2=- hip2=-=KWOK_HOST_ALLOC=hip > /dev/null || exit 4
for v in reg hip reg2 hip2; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
cd /tmp && export TMPDIR=/tmp
KWOK_HOST_ALLOC=hip timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/prof_s39 -o run -- python3 $R/tools/c4_probe.py --ticks 3 --together --once > $R/gpurun_out/prof_s39.log 2>&1 || exit 5
T=$(find $R/gpurun_out/prof_s39 -name 'run_kernel_trace.csv' | head -n 1)
M=$(find $R/gpurun_out/prof_s39 -name 'run_memory_copy_trace.csv' | head -n 1)
python3 $R/tools/timeline.py "$T" --last 22 --copies "$M" > $R/gpurun_out/timeline_s39.txt
cat $R/gpurun_out/timeline_s39.txt
