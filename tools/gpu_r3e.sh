#!/bin/bash
# Round-3 checkpoint C: GPU suite (parallel apply path), bench with the ingest
# split, and the C5 flap leg with single-threaded node ingest (A/B).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3e_tests.log 2>&1
rc=$?
tail -4 $R/gpurun_out/r3e_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3e_tests.log | head -30; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/r3e_bench.json 2> $R/gpurun_out/r3e_bench.err || { tail -20 $R/gpurun_out/r3e_bench.err; exit 3; }
KWOK_INGEST_PROF=1 KWOK_NODE_PAR_MIN=100000000 timeout -k 10 400 python bench.py --steps 10 --churn-ticks 0 --cpu-baseline 0 --roofline-ticks 0 > $R/gpurun_out/r3e_flap1.json 2> $R/gpurun_out/r3e_flap1.err || exit 4
cut -c1-300 $R/gpurun_out/r3e_bench.json
exit 0
