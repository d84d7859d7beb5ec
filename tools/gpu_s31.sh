# the copy form of the create handles whenever a tick is queued behind the batch:
# the batch-with-tick parity tests (all sizes), then the C4 A/B leg once more
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ingest_tick_gpu.py \
  tests/test_c4_churn_gpu.py tests/test_ingest_chunks_gpu.py > gpurun_out/s31_tests.txt 2>&1 || { tail -30 gpurun_out/s31_tests.txt; exit 3; }
tail -1 gpurun_out/s31_tests.txt
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh new=- new2=- > /dev/null || exit 4
for v in new new2; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
