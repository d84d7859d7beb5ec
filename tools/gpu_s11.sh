set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_c4_churn_gpu.py tests/test_once_gpu.py tests/test_emit_paths_gpu.py -k "not metric_size or drop_in" > gpurun_out/s11_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s11_tests.log; [ $rc -eq 0 ] || exit 3
V=kwok_amd/lib/var
bash tools/gpu_c4ab.sh s11 rows2= rows1=KWOK_ENGINE_LIB=$V/libkwok_engine_rows1.so rows3=KWOK_ENGINE_LIB=$V/libkwok_engine_rows3.so rows2b= rows1b=KWOK_ENGINE_LIB=$V/libkwok_engine_rows1.so || exit 4
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=3 timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 3 > gpurun_out/s11_trace.json 2> gpurun_out/s11_trace.err || { tail -5 gpurun_out/s11_trace.err; exit 5; }
grep "kwok trace\]" gpurun_out/s11_trace.err | tail -22
