set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_json_nodes_gpu.py tests/test_json_gpu.py tests/test_c5_flap_gpu.py tests/test_controller_gpu.py > gpurun_out/s14_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s14_tests.log; [ $rc -eq 0 ] || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_s14 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --leg flap_once --flap-ticks 3 > $GRAFT_REPO_ROOT/gpurun_out/s14_flap.json 2>/dev/null || exit 4
grep json $GRAFT_REPO_ROOT/gpurun_out/prof_s14/*/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/prof_s14/run_kernel_stats.csv 2>/dev/null
python3 -c "import json; d=json.loads(open('$GRAFT_REPO_ROOT/gpurun_out/s14_flap.json').read().strip().splitlines()[-1]); print(d['from_json'])"
