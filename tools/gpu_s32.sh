# is the k_tick slowdown beside the batch's result copies the blit kernels'
# workgroups?  C4 (tick behind the batch, heartbeat-once engine) with the runtime's
# blit kernels limited to 4 / 1 workgroups (DEBUG_CLR_LIMIT_BLIT_WG) against the default,
# then a kernel trace with 1
set -o pipefail
R=$GRAFT_REPO_ROOT
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh d=- w4=-=DEBUG_CLR_LIMIT_BLIT_WG=4 w1=-=DEBUG_CLR_LIMIT_BLIT_WG=1 d2=- w1b=-=DEBUG_CLR_LIMIT_BLIT_WG=1 > /dev/null || exit 4
for v in d w4 w1 d2 w1b; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
cd /tmp && export TMPDIR=/tmp
for v in 16 1; do
DEBUG_CLR_LIMIT_BLIT_WG=$v timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/prof_s32_$v -o run -- python3 $R/tools/c4_probe.py --ticks 3 --together --once > $R/gpurun_out/prof_s32_$v.log 2>&1 || exit 5
T=$(find $R/gpurun_out/prof_s32_$v -name 'run_kernel_trace.csv' | head -n 1)
M=$(find $R/gpurun_out/prof_s32_$v -name 'run_memory_copy_trace.csv' | head -n 1)
python3 $R/tools/timeline.py "$T" --last 22 --copies "$M" > $R/gpurun_out/timeline_s32_$v.txt
echo "== $v"; cat $R/gpurun_out/timeline_s32_$v.txt
python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
print('columns', list(rows[0].keys())[:40])
for r in rows[-12:]:
  if 'copyBuffer' in r['Kernel_Name']: print(r['Kernel_Name'][:40], r.get('Grid_Size_X', r.get('Grid_Size')), r.get('Workgroup_Size_X', r.get('Workgroup_Size')))
" "$T"
done
