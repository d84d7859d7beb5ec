#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $R/tests/test_c4_churn_gpu.py $R/tests/test_ingest_chunks_gpu.py $R/tests/test_parity_gpu.py $R/tests/test_controller_gpu.py > $R/gpurun_out/r4q_t.log 2>&1
rc=$?; tail -2 $R/gpurun_out/r4q_t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/r4q_t.log | head -20; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 300 python3 -u $R/tools/stall_probe.py 40 > $R/gpurun_out/r4q.txt 2> $R/gpurun_out/r4q.err || { tail -5 $R/gpurun_out/r4q.err; exit 4; }
grep step $R/gpurun_out/r4q.txt | awk '{print $4}' | tr '\n' ' '; echo
grep -E "wait for its prep|records at \+[2-9]" $R/gpurun_out/r4q.err | tail -5
