set -o pipefail
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=3 timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 4 > gpurun_out/s3_trace.json 2> gpurun_out/s3_trace.err || exit 1
grep "kwok trace" gpurun_out/s3_trace.err
bash tools/gpu_c4ab.sh s3 lean= || exit 2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_controller_gpu.py tests/test_c4_churn_gpu.py tests/test_once_gpu.py > gpurun_out/s3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s3_tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python -u bench.py --leg hb_once --steps 20 --churn-ticks 3 --json-ticks 1 > gpurun_out/s3_hbonce.json 2> gpurun_out/s3_hbonce.err || { tail -20 gpurun_out/s3_hbonce.err; exit 4; }
python3 -c "
import json; d=json.loads(open('gpurun_out/s3_hbonce.json').read().strip().splitlines()[-1])
print(json.dumps(d['initial_tick'])[:900]); print(json.dumps(d['churn'])[:2500])"
