#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $R/tests/test_ingest_chunks_gpu.py $R/tests/test_growth_gpu.py $R/tests/test_c4_churn_gpu.py $R/tests/test_parity_gpu.py $R/tests/test_controller_gpu.py $R/tests/test_dist_gpu.py $R/tests/test_rccl_gpu.py $R/tests/test_cni_gpu.py $R/tests/test_use_checks_gpu.py > $R/gpurun_out/r4s_t.log 2>&1
rc=$?; tail -2 $R/gpurun_out/r4s_t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/r4s_t.log | head -20; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 300 python3 -u $R/tools/stall_probe.py 30 > $R/gpurun_out/r4s.txt 2> $R/gpurun_out/r4s.err || { tail -5 $R/gpurun_out/r4s.err; exit 4; }
grep step $R/gpurun_out/r4s.txt | awk '{print $4, $7}' | tr '\n' ' '; echo
grep -E "queued and applied" $R/gpurun_out/r4s.err | tail -3
