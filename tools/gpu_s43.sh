# k_nd_apply with the bucket's first 64 node records loaded together ahead of its
# serial loop: the node-ingest parity tests, then C5 (records and documents) against
# the previous build (prev) with k_nd_apply's trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_node_dir_gpu.py tests/test_c5_flap_gpu.py \
  tests/test_parity_gpu.py tests/test_json_nodes_gpu.py tests/test_ingest_chunks_gpu.py tests/test_controller_gpu.py tests/test_dist_gpu.py > gpurun_out/s43_tests.txt 2>&1 || { tail -30 gpurun_out/s43_tests.txt; exit 3; }
tail -1 gpurun_out/s43_tests.txt
for v in prev new prev new; do
  L=$R/kwok_amd/lib/libkwok_engine.so; [ $v = prev ] && L=$R/kwok_amd/lib/var/libkwok_engine_prev.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 python -u bench.py --leg flap_once --flap-ticks 8 > gpurun_out/s43_$v.json 2> gpurun_out/s43_$v.err || { tail -5 gpurun_out/s43_$v.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'C5 records %.3f (ingest %.3f) json %.3f' % (d['ms_per_step'], d['ingest_ms'], d['from_json']['ms_per_step']))" gpurun_out/s43_$v.json $v
done
cd /tmp && export TMPDIR=/tmp
for v in prev new; do
  L=$R/kwok_amd/lib/libkwok_engine.so; [ $v = prev ] && L=$R/kwok_amd/lib/var/libkwok_engine_prev.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s43_$v -o run -- python3 $R/bench.py --leg flap_once --flap-ticks 6 > $R/gpurun_out/prof_s43_$v.log 2>&1 || exit 5
  T=$(find $R/gpurun_out/prof_s43_$v -name 'run_kernel_trace.csv' | head -n 1)
  python3 $R/tools/trace_summary.py "$T" --last 6 --out $R/gpurun_out/ktrace_s43_$v.txt
  echo "== $v $(grep -E 'k_nd_apply' $R/gpurun_out/ktrace_s43_$v.txt)"
done
