set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_json_nodes_gpu.py tests/test_json_gpu.py tests/test_c5_flap_gpu.py > gpurun_out/s8_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s8_tests.log; [ $rc -eq 0 ] || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_s8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --leg flap_once --flap-ticks 3 > $GRAFT_REPO_ROOT/gpurun_out/s8_flap.json 2>/dev/null || exit 4
T=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_s8 -name run_kernel_trace.csv | head -1); python3 $GRAFT_REPO_ROOT/tools/timeline.py $T --last 30 | grep json
python3 -c "import json; d=json.loads(open('$GRAFT_REPO_ROOT/gpurun_out/s8_flap.json').read().strip().splitlines()[-1]); print(d['from_json'])"
cd $GRAFT_REPO_ROOT && KWOK_INGEST_PROF=1 timeout -k 10 600 python -u bench.py --leg hb_once --steps 10 --churn-ticks 2 --json-ticks 2 > gpurun_out/s8_hb.json 2> gpurun_out/s8_hb.err || exit 5
grep "kwok json" gpurun_out/s8_hb.err | tail -4
python3 -c "import json; d=json.loads(open('gpurun_out/s8_hb.json').read().strip().splitlines()[-1]); c=d['churn_json']; print(c['ms_per_step'], c['decode_ingest_ms'], c['documents_per_s'])"
cd $GRAFT_REPO_ROOT && timeout -k 10 900 python -u -m pytest -x -q --timeout 880 --timeout-method thread -m gpu tests/test_c4_churn_gpu.py -k drop_in > gpurun_out/s8_c4.log 2>&1; rc=$?; tail -3 gpurun_out/s8_c4.log; exit $rc
