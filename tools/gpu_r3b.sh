#!/bin/bash
# Round-3 checkpoint B: the whole GPU suite (GPU pod ingest), then the default
# bench with the ingest phase split on stderr.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3b_tests.log 2>&1
rc=$?
tail -4 $R/gpurun_out/r3b_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3b_tests.log | head -30; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --cpu-baseline 0 > $R/gpurun_out/r3b_bench.json 2> $R/gpurun_out/r3b_bench.err || { tail -20 $R/gpurun_out/r3b_bench.err; exit 3; }
cut -c1-300 $R/gpurun_out/r3b_bench.json
exit 0
