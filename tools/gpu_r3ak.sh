#!/bin/bash
# Node ingest with software-prefetched name lookups: C5 / parity GPU tests, then the
# C5 flap leg A/B over the prefetch distance (KWOK_NODE_PF; 0 = next to none).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 400 --timeout-method thread tests/test_c5_flap_gpu.py tests/test_parity_gpu.py tests/test_growth_gpu.py > $R/gpurun_out/rak_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/rak_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/rak_tests.log | head -30; exit $rc; }
for pf in 0 16 24 0 16 24; do
  KWOK_NODE_PF=$pf KWOK_INGEST_PROF=1 timeout -k 10 300 python bench.py --steps 10 --churn-ticks 0 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 8 > $R/gpurun_out/rak_flap$pf.json 2> $R/gpurun_out/rak_flap$pf.err || exit 2
  python3 -c "import json; f=json.load(open('$R/gpurun_out/rak_flap$pf.json'))['flap']; print('pf $pf: step %.3f ingest %.3f tick %.3f' % (f['ms_per_step'], f['ingest_ms'], f['tick_ms']))"
  grep "9990 node" $R/gpurun_out/rak_flap$pf.err | tail -3
done
exit 0
