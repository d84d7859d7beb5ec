# C4 ingest at 1..4 chunks per 2M-record batch (KWOK_INGEST_CHUNK), main leg only
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
for C in 2000000 1000000 700000 500000; do
  KWOK_INGEST_CHUNK=$C KWOK_INGEST_PROF=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --churn-ticks 8 --flap-ticks 0 --emulate-ranks 0 --c2 0 --json-ticks 0 --roofline-ticks 0 > $R/gpurun_out/chunk_${TAG}_$C.json 2> $R/gpurun_out/chunk_${TAG}_$C.err || { tail -20 $R/gpurun_out/chunk_${TAG}_$C.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$R/gpurun_out/chunk_${TAG}_$C.json') if l.startswith('{')][-1]); c=d['churn']
print($C, {k: round(c[k],3) for k in ('ms_per_step','ingest_ms','tick_ms')}, c['median_ms'])"
  grep "device from chunk" $R/gpurun_out/chunk_${TAG}_$C.err | tail -2
done
