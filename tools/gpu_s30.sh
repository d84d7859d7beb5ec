# kwok_pod_rec12's create handles written in place by the kernel (default) or
# into HBM and copied back (KWOK_INGEST_NEW_MAPPED=0): C4 on the heartbeat-once
# engine, with the tick behind the batch and as two calls, each three times alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh t1a=- t0a=-=KWOK_INGEST_NEW_MAPPED=0 t1b=- t0b=-=KWOK_INGEST_NEW_MAPPED=0 t1c=- t0c=-=KWOK_INGEST_NEW_MAPPED=0 > /dev/null || exit 4
C4ARGS="--once" bash $R/tools/gpu_c4_ab.sh s1a=- s0a=-=KWOK_INGEST_NEW_MAPPED=0 s1b=- s0b=-=KWOK_INGEST_NEW_MAPPED=0 > /dev/null || exit 5
for v in t1a t0a t1b t0b t1c t0c s1a s0a s1b s0b; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
