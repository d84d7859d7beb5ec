# the last apply pass writes the tick's skip flag (no device-to-device copy launch
# between it and the tick): the batch-with-tick parity tests (growth cases included),
# then C4 A/B against the previous build (prev)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ingest_tick_gpu.py \
  tests/test_c4_churn_gpu.py -k "tick or together or growth" > gpurun_out/s33_tests.txt 2>&1 || { tail -30 gpurun_out/s33_tests.txt; exit 3; }
tail -1 gpurun_out/s33_tests.txt
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh prev=$R/kwok_amd/lib/var/libkwok_engine_prev.so new=- prev2=$R/kwok_amd/lib/var/libkwok_engine_prev.so new2=- > /dev/null || exit 4
for v in prev new prev2 new2; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
