#!/bin/bash
for NG in 0 1; do
  KWOK_NO_GRAPH=$NG timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_ng$NG.json 2>/dev/null || exit $?
  KWOK_NO_GRAPH=$NG timeout -k 10 300 python bench.py --nodes-per-rank 1000 --cpu-baseline 0 > gpurun_out/bench_ng${NG}_floor.json 2>/dev/null || exit $?
done
for f in gpurun_out/bench_ng0.json gpurun_out/bench_ng0_floor.json gpurun_out/bench_ng1.json gpurun_out/bench_ng1_floor.json; do echo $f; cat $f; done
