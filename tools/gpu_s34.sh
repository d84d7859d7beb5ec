# documents per wave in the JSON scanners (KWOK_JSON_NODE_LANES / KWOK_JSON_POD_LANES):
# the device codec tests at 16 lanes, then C5 from its node documents at 64 / 32 / 16 / 8
# lanes, with k_json_nodes' kernel time from a trace at 64 and 16
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
KWOK_JSON_NODE_LANES=16 KWOK_JSON_POD_LANES=16 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_json_gpu.py tests/test_json_nodes_gpu.py > gpurun_out/s34_tests.txt 2>&1 || { tail -30 gpurun_out/s34_tests.txt; exit 3; }
tail -1 gpurun_out/s34_tests.txt
for L in 64 32 16 8 64 16; do
  KWOK_JSON_NODE_LANES=$L timeout -k 10 300 python -u bench.py --leg flap_once --flap-ticks 8 > gpurun_out/s34_$L.json 2> gpurun_out/s34_$L.err || { tail -5 gpurun_out/s34_$L.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lanes', sys.argv[2], 'records %.3f json %.3f' % (d['ms_per_step'], d['from_json']['ms_per_step']))" gpurun_out/s34_$L.json $L
done
cd /tmp && export TMPDIR=/tmp
for L in 64 16; do
  KWOK_JSON_NODE_LANES=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s34_$L -o run -- python3 $R/bench.py --leg flap_once --flap-ticks 4 > $R/gpurun_out/prof_s34_$L.log 2>&1 || exit 5
  T=$(find $R/gpurun_out/prof_s34_$L -name 'run_kernel_trace.csv' | head -n 1)
  python3 $R/tools/trace_summary.py "$T" --last 4 --out $R/gpurun_out/ktrace_s34_$L.txt
  echo "== $L"; grep -E "k_json" $R/gpurun_out/ktrace_s34_$L.txt
done
