#!/bin/bash
# Rehearsal of the driver's N>1 bench on the one-GPU box: two ranks on GPU 0, the
# exchange over the host allgather hook (KWOK_BENCH_REHEARSAL=1; RCCL refuses two
# ranks on one GPU), default legs (churn on every rank with the exchange time).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
KWOK_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 > $R/gpurun_out/raj_n2.json 2> $R/gpurun_out/raj_n2.err || { tail -30 $R/gpurun_out/raj_n2.err; exit 2; }
cut -c1-1500 $R/gpurun_out/raj_n2.json
exit 0
