#!/bin/bash
# N=2 bench rehearsal on one GPU (host-memory exchange over gloo; never a reported number)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
KWOK_BENCH_REHEARSAL=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 10 --warmup 2 --churn-ticks 3 > $R/gpurun_out/r4z.json 2> $R/gpurun_out/r4z.err || { tail -20 $R/gpurun_out/r4z.err; exit 4; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/r4z.json'))
print({k: d[k] for k in ('value','ms_per_step','n_gpus','scaling')})
c=d.get('churn'); print('churn', c and {k: c[k] for k in ('ms_per_step','ingest_ms','tick_ms','exchange_ms','steps_ms')})
"
