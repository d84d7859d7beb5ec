#!/bin/bash
# Round-3 checkpoint AC: chunked pod ingest (chunk k+1's prep over the link
# beside chunk k's apply and result copies).  Ingest GPU tests, C4 churn A/B over
# the chunk size, the 7.2 GB fill ceiling (k_emit's initial-tick write volume).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_ingest_chunks_gpu.py tests/test_c4_churn_gpu.py tests/test_growth_gpu.py tests/test_use_checks_gpu.py > $R/gpurun_out/rac_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/rac_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/rac_tests.log | head -30; exit $rc; }
for ch in 100000000 1048576 524288 393216; do
  KWOK_INGEST_CHUNK=$ch KWOK_INGEST_PROF=1 timeout -k 10 300 python bench.py --steps 10 --churn-ticks 6 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 0 > $R/gpurun_out/rac_churn$ch.json 2> $R/gpurun_out/rac_churn$ch.err || exit 2
  python3 -c "import json; c=json.load(open('$R/gpurun_out/rac_churn$ch.json'))['churn']; print('chunk $ch: step %.3f (median %.3f) ingest %.3f (median %.3f) tick %.3f' % (c['ms_per_step'], c['median_ms']['step'], c['ingest_ms'], c['median_ms']['ingest'], c['tick_ms']))"
  grep "kwok ingest" $R/gpurun_out/rac_churn$ch.err | tail -6
done
exit 0
