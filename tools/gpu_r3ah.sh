#!/bin/bash
# Multi-rank stream tail (the chain blocks' share of the heartbeat stream as its own
# launch beside the exchange + BACK): multi-rank GPU tests, chunked-ingest tests,
# then the one-rank RCCL tick (KWOK_FORCE_MULTI=1) with and without the tail, and the
# single-rank default.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_ingest_chunks_gpu.py tests/test_rccl_gpu.py tests/test_dist_gpu.py tests/test_dist_scale_gpu.py tests/test_c3_8rank_gpu.py > $R/gpurun_out/rah_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/rah_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/rah_tests.log | head -30; exit $rc; }
for v in "tail1:KWOK_FORCE_MULTI=1" "tail0:KWOK_FORCE_MULTI=1 KWOK_TICK_TAIL=0" "tail1b:KWOK_FORCE_MULTI=1" "tail0b:KWOK_FORCE_MULTI=1 KWOK_TICK_TAIL=0" "s900:KWOK_FORCE_MULTI=1 KWOK_TICK_STREAM_SHARE=900" "s820:KWOK_FORCE_MULTI=1 KWOK_TICK_STREAM_SHARE=820" "single:KWOK_X=0"; do
  n=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --steps 100 --warmup 5 --cpu-baseline 0 --roofline-ticks 20 --churn-ticks 3 --flap-ticks 0 --once-ticks 0 > $R/gpurun_out/rah_$n.json 2> $R/gpurun_out/rah_$n.err || { tail -5 $R/gpurun_out/rah_$n.err; exit 2; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/rah_$n.json')); c=d['churn']; print('%-7s step %.4f ms  churn step %.3f tick %.3f exchange %s' % ('$n', d['ms_per_step'], c['ms_per_step'], c['tick_ms'], c.get('exchange_ms')))"
done
exit 0
