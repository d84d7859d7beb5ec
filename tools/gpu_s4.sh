set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_json_nodes_gpu.py tests/test_c5_flap_gpu.py tests/test_controller_gpu.py tests/test_json_gpu.py > gpurun_out/s4_tests.log 2>&1; rc=$?; tail -15 gpurun_out/s4_tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python -u bench.py --leg flap_once --flap-ticks 5 > gpurun_out/s4_flap.json 2> gpurun_out/s4_flap.err || { tail -20 gpurun_out/s4_flap.err; exit 4; }
tail -c 1500 gpurun_out/s4_flap.json
timeout -k 10 600 python -u bench.py --leg hb_once --steps 20 --churn-ticks 3 --json-ticks 2 > gpurun_out/s4_hbonce.json 2> gpurun_out/s4_hbonce.err || { tail -20 gpurun_out/s4_hbonce.err; exit 5; }
python3 -c "
import json; d=json.loads(open('gpurun_out/s4_hbonce.json').read().strip().splitlines()[-1])
print(json.dumps(d['churn']['with_handoff'])); print(json.dumps(d['churn_json'])[:1500])"
