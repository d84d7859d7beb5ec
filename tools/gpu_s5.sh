set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_once_gpu.py tests/test_parity_gpu.py tests/test_controller_gpu.py tests/test_custom_template_gpu.py > gpurun_out/s5_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s5_tests.log; [ $rc -eq 0 ] || exit 3
bash tools/gpu_c4ab.sh s5 nostream= || exit 4
for RS in 1 2 4; do
  KWOK_READ_STREAMS=$RS timeout -k 10 600 python -u bench.py --leg hb_once --steps 20 --churn-ticks 3 --json-ticks 0 > gpurun_out/s5_rs$RS.json 2> gpurun_out/s5_rs$RS.err || { tail -20 gpurun_out/s5_rs$RS.err; exit 5; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s5_rs$RS.json').read().strip().splitlines()[-1])
i=d['initial_tick']['with_handoff']; h=d['churn']['with_handoff']
print('RS=$RS init read %.1f ms %.1f GB/s; c4 seq %.2f ms (%.1f GB/s) ovl %.2f ms; c4 kernel %.3f' % (i['read_ms'], i['link_gbs'], h['sequential']['ms_per_step'], h['sequential']['link_gbs_equivalent'], h['overlapped']['ms_per_step'], d['churn']['kernel_ms']))"
done
