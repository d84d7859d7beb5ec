# k_json_nodes without scratch memory (its scan state had been kept in scratch: the
# 16-byte window's byte pick compiled to an indexed load, and the nodeInfo spans
# were indexed): the node codec tests (golden, mutated, fuzzed, C5 from documents),
# then C5 from its node documents by documents per wave, and k_json_nodes' trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_json_nodes_gpu.py tests/test_json_gpu.py \
  tests/test_json_fuzz_gpu.py tests/test_c5_flap_gpu.py > gpurun_out/s35_tests.txt 2>&1 || { tail -30 gpurun_out/s35_tests.txt; exit 3; }
tail -1 gpurun_out/s35_tests.txt
for L in 64 32 16 64; do
  KWOK_JSON_NODE_LANES=$L timeout -k 10 300 python -u bench.py --leg flap_once --flap-ticks 8 > gpurun_out/s35_$L.json 2> gpurun_out/s35_$L.err || { tail -5 gpurun_out/s35_$L.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lanes', sys.argv[2], 'records %.3f json %.3f' % (d['ms_per_step'], d['from_json']['ms_per_step']))" gpurun_out/s35_$L.json $L
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s35 -o run -- python3 $R/bench.py --leg flap_once --flap-ticks 4 > $R/gpurun_out/prof_s35.log 2>&1 || exit 5
T=$(find $R/gpurun_out/prof_s35 -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 4 --out $R/gpurun_out/ktrace_s35.txt
grep -E "k_json|k_nd_" $R/gpurun_out/ktrace_s35.txt
