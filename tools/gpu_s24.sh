# C4 churn (the tick behind the batch) by KWOK_INGEST_CHUNK, after the faster
# scatter: 1M (default), 700k (3 chunks), 512k (4), 400k (5), default again
set -o pipefail
R=$GRAFT_REPO_ROOT
C4ARGS=--together bash $R/tools/gpu_c4_ab.sh c1m=- c700k=-=KWOK_INGEST_CHUNK=700000 c512k=-=KWOK_INGEST_CHUNK=524288 \
  c400k=-=KWOK_INGEST_CHUNK=400000 c1mb=- c700kb=-=KWOK_INGEST_CHUNK=700000 || exit 4
for v in c1m c700k c512k c400k c1mb c700kb; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
