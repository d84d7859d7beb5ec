# a chunked pod batch's H2D copies on their own stream (engine.cpp prep): the
# ingest parity tests, then C4 (the tick behind the batch, heartbeat-once engine)
# with the copies on the prep stream (KWOK_INGEST_CS=0) and on their own, at 1M-
# and 512k-record chunks
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingest_chunks_gpu.py \
  tests/test_ingest_tick_gpu.py tests/test_c4_churn_gpu.py tests/test_growth_gpu.py > gpurun_out/s26_tests.txt 2>&1 || { tail -30 gpurun_out/s26_tests.txt; exit 3; }
tail -1 gpurun_out/s26_tests.txt
C4ARGS="--together --once" bash tools/gpu_c4_ab.sh ps1m=-=KWOK_INGEST_CS=0 cs1m=- ps512k=-=KWOK_INGEST_CS=0,KWOK_INGEST_CHUNK=524288 \
  cs512k=-=KWOK_INGEST_CHUNK=524288 cs700k=-=KWOK_INGEST_CHUNK=700000 ps1mb=-=KWOK_INGEST_CS=0 cs1mb=- > /dev/null || exit 4
for v in ps1m cs1m ps512k cs512k cs700k ps1mb cs1mb; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
