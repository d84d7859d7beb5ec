#!/bin/bash
# new GPU tests (drop-in controller, ingest poisoning), then the heartbeat-once probe + trace
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest $R/tests/test_controller_gpu.py $R/tests/test_ingest_chunks_gpu.py -x -v --timeout 600 --timeout-method thread > $R/gpurun_out/r4c_tests.log 2>&1
rc=$?; tail -15 $R/gpurun_out/r4c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 $R/tools/once_probe.py 100 base > $R/gpurun_out/r4c.txt 2> $R/gpurun_out/r4c.err || { tail -5 $R/gpurun_out/r4c.err; exit 2; }
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=8 timeout -k 10 120 python3 $R/tools/once_probe.py 50 trace >> $R/gpurun_out/r4c.txt 2> $R/gpurun_out/r4c_trace.err || { tail -5 $R/gpurun_out/r4c_trace.err; exit 3; }
cat $R/gpurun_out/r4c.txt; grep "kwok trace" $R/gpurun_out/r4c_trace.err
