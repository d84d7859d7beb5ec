#!/bin/bash
# Round-3 checkpoint Z: node ingest partitions keep their accumulators and
# per-record results on cache lines of their own.  GPU suite, C5 flap at 16 / 4
# partition threads.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r3z_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/r3z_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/r3z_tests.log | head -30; exit $rc; }
for th in 16 4; do
  KWOK_INGEST_THREADS=$th KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 10 --churn-ticks 0 --cpu-baseline 0 --roofline-ticks 0 --once-ticks 0 --flap-ticks 8 > $R/gpurun_out/r3z_flap$th.json 2> $R/gpurun_out/r3z_flap$th.err || exit 2
  grep "9990 node" $R/gpurun_out/r3z_flap$th.err | tail -2
  python3 -c "import json; f=json.load(open('$R/gpurun_out/r3z_flap$th.json'))['flap']; print('threads $th: step %.3f ingest %.3f tick %.3f' % (f['ms_per_step'], f['ingest_ms'], f['tick_ms']))"
done
exit 0
