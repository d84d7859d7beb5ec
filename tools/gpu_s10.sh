set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_c4_churn_gpu.py tests/test_once_gpu.py tests/test_use_checks_gpu.py tests/test_emit_paths_gpu.py -k "not metric_size or drop_in" > gpurun_out/s10_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s10_tests.log; [ $rc -eq 0 ] || exit 3
bash tools/gpu_c4ab.sh s10 bytes= atomics=KWOK_REL_BYTES=0 bytes2= atomics2=KWOK_REL_BYTES=0 || exit 4
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=3 KWOK_TICK_TRACE_SLOW=1 timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 3 > gpurun_out/s10_trace.json 2> gpurun_out/s10_trace.err || { tail -5 gpurun_out/s10_trace.err; exit 5; }
grep "kwok trace" gpurun_out/s10_trace.err | tail -30
