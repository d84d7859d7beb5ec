# k_ing_apply (records fetched one chunk ahead, bitmap loads unrolled) and
# k_bs_scatter (W waves per tile): the ingest parity tests, then the C4 churn A/B
# (the tick behind the batch) against the round-6 ingest (base), with kernel traces
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingest_chunks_gpu.py tests/test_json_gpu.py tests/test_node_dir_gpu.py \
  tests/test_ingest_tick_gpu.py tests/test_c4_churn_gpu.py tests/test_growth_gpu.py tests/test_parity_gpu.py tests/test_c5_flap_gpu.py > gpurun_out/s23_tests.txt 2>&1 || { tail -30 gpurun_out/s23_tests.txt; exit 3; }
tail -3 gpurun_out/s23_tests.txt
C4ARGS=--together bash tools/gpu_c4_ab.sh base=$R/kwok_amd/lib/var/libkwok_engine_base.so new=- base2=$R/kwok_amd/lib/var/libkwok_engine_base.so new2=- || exit 4
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  L=$R/kwok_amd/lib/libkwok_engine.so; [ $v = base ] && L=$R/kwok_amd/lib/var/libkwok_engine_base.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s23_$v -o run -- python3 $R/tools/c4_probe.py --ticks 3 --together > $R/gpurun_out/prof_s23_$v.log 2>&1 || exit 5
  T=$(find $R/gpurun_out/prof_s23_$v -name 'run_kernel_trace.csv' | head -n 1)
  python3 $R/tools/trace_summary.py "$T" --last 3 --out $R/gpurun_out/ktrace_s23_$v.txt
  echo "== $v"; grep -E "k_ing|k_bs|k_tick|k_emit" $R/gpurun_out/ktrace_s23_$v.txt | head -12
done
