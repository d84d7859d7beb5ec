# the JSON scanners with 32-bit positions: the device codec tests (pods and nodes:
# golden, mutated, fuzzed, C5 and the controller through them), then k_json_nodes /
# k_json_pods kernel times (C5 from node documents; C4 from pod documents)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_json_nodes_gpu.py tests/test_json_gpu.py \
  tests/test_json_fuzz_gpu.py tests/test_c5_flap_gpu.py tests/test_controller_gpu.py > gpurun_out/s37_tests.txt 2>&1 || { tail -30 gpurun_out/s37_tests.txt; exit 3; }
tail -1 gpurun_out/s37_tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s37 -o run -- python3 $R/bench.py --leg flap_once --flap-ticks 6 > $R/gpurun_out/prof_s37.log 2>&1 || exit 5
T=$(find $R/gpurun_out/prof_s37 -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 6 --out $R/gpurun_out/ktrace_s37.txt
grep -E "k_json" $R/gpurun_out/ktrace_s37.txt
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C5 records %.3f json %.3f' % (d['ms_per_step'], d['from_json']['ms_per_step']))" $R/gpurun_out/prof_s37.log || true
