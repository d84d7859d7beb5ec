#!/bin/bash
# device node directory (GPU node ingest, by-name pods resolved in the apply pass):
# node / pod parity tests, then the rest of the GPU suite, C5 flap leg, multi-rank spec A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
T="python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T $R/tests/test_parity_gpu.py $R/tests/test_ingest_chunks_gpu.py $R/tests/test_c5_flap_gpu.py $R/tests/test_controller_gpu.py $R/tests/test_custom_template_gpu.py $R/tests/test_cni_gpu.py $R/tests/test_growth_gpu.py > $R/gpurun_out/r4i_t1.log 2>&1
rc=$?; tail -3 $R/gpurun_out/r4i_t1.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/r4i_t1.log | head -30; exit $rc; }
KWOK_INGEST_PROF=1 timeout -k 10 300 python3 $R/bench.py --steps 20 --cpu-baseline 0 --churn-ticks 0 --once-ticks 0 --emulate-ranks 0 --flap-ticks 10 > $R/gpurun_out/r4i_flap.json 2> $R/gpurun_out/r4i_flap.err || { tail -5 $R/gpurun_out/r4i_flap.err; exit 4; }
python3 -c "import json; d=json.load(open('$R/gpurun_out/r4i_flap.json')); print('steady', d['ms_per_step']); print('flap', json.dumps(d['flap']))"
grep "node records" $R/gpurun_out/r4i_flap.err | tail -4
timeout -k 10 900 $T $R/tests/test_dist_gpu.py $R/tests/test_rccl_gpu.py $R/tests/test_c3_8rank_gpu.py $R/tests/test_use_checks_gpu.py $R/tests/test_emit_paths_gpu.py $R/tests/test_c4_churn_gpu.py $R/tests/test_dist_scale_gpu.py > $R/gpurun_out/r4i_t2.log 2>&1
rc=$?; tail -3 $R/gpurun_out/r4i_t2.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/r4i_t2.log | head -30; exit $rc; }
for X in 0 1; do
KWOK_XSPEC=$((X*256)) KWOK_FORCE_MULTI=1 timeout -k 10 300 python3 $R/bench.py --steps 30 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --churn-ticks 3 --emulate-ranks 8 > $R/gpurun_out/r4i_multi$X.json 2> $R/gpurun_out/r4i_multi$X.err || { tail -5 $R/gpurun_out/r4i_multi$X.err; exit 5; }
python3 - $R/gpurun_out/r4i_multi$X.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], 'steady', d['ms_per_step'], 'k_tick', d['roofline']['avg_launch_ms'])
for k in ('churn', 'churn_events'):
    c = d.get(k)
    if c: print(' ', k, json.dumps(c))
print('  emulated', json.dumps(d.get('emulated_ranks')))
PY
done
