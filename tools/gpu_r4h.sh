#!/bin/bash
# multi-rank list segments + once prefetch: GPU tests; steady-tick variant A/B; one-rank RCCL churn
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 1100 python -u -m pytest $R/tests/test_dist_gpu.py $R/tests/test_rccl_gpu.py $R/tests/test_controller_gpu.py $R/tests/test_parity_gpu.py $R/tests/test_c3_8rank_gpu.py -m gpu -x -v --timeout 1100 --timeout-method thread > $R/gpurun_out/r4h_tests.log 2>&1
rc=$?; tail -3 $R/gpurun_out/r4h_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/r4h_tests.log | head -30; exit $rc; }
: > $R/gpurun_out/r4h.txt
for V in def orig def orig; do
  L=$R/kwok_amd/lib/var/libkwok_engine_$V.so; [ $V = def ] && L=$R/kwok_amd/lib/libkwok_engine.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 100 --cpu-baseline 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 > $R/gpurun_out/r4h_b.json 2> $R/gpurun_out/r4h_b.err || { tail -5 $R/gpurun_out/r4h_b.err; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'steady', round(d['ms_per_step'],4), 'k_tick', round(d['roofline']['avg_launch_ms'],4), 'classify', round(d['state_only']['classify_ms'],4))" $R/gpurun_out/r4h_b.json $V >> $R/gpurun_out/r4h.txt
done
KWOK_XSPEC=0 KWOK_FORCE_MULTI=1 timeout -k 10 300 python3 $R/bench.py --steps 30 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --churn-ticks 3 --emulate-ranks 8 > $R/gpurun_out/r4h_multi0.json 2> $R/gpurun_out/r4h_multi0.err || { tail -5 $R/gpurun_out/r4h_multi0.err; exit 5; }
KWOK_FORCE_MULTI=1 timeout -k 10 300 python3 $R/bench.py --steps 30 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --churn-ticks 3 --emulate-ranks 8 > $R/gpurun_out/r4h_multi.json 2> $R/gpurun_out/r4h_multi.err || { tail -5 $R/gpurun_out/r4h_multi.err; exit 5; }
python3 - >> $R/gpurun_out/r4h.txt <<'PY'
import json
for f in ('r4h_multi0', 'r4h_multi'):
    d=json.load(open('/root/repo/gpurun_out/%s.json' % f))
    print(f, 'steady', d['ms_per_step'], 'k_tick', d['roofline']['avg_launch_ms'])
    for k in ('churn','churn_events'):
        c=d.get(k)
        if c: print(' ', k, json.dumps(c))
    print('  emulated', json.dumps(d.get('emulated_ranks')))
PY
cat $R/gpurun_out/r4h.txt
