#!/bin/bash
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_r1g.json 2>gpurun_out/bench_r1g.err || exit $?
timeout -k 10 300 python bench.py --nodes-per-rank 1000 --cpu-baseline 0 > gpurun_out/bench_r1g_floor.json 2>/dev/null || exit $?
cat gpurun_out/bench_r1g.json gpurun_out/bench_r1g_floor.json
