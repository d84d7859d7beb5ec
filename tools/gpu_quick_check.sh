set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $R/gpurun_out/tests_q.log 2>&1; rc=$?; tail -3 $R/gpurun_out/tests_q.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $R/gpurun_out/tests_q.log | head; exit $rc; }
timeout -k 10 200 python bench.py --steps 50 --warmup 3 --cpu-baseline 0 --roofline-ticks 0 --churn-ticks 0 --flap-ticks 0 > $R/gpurun_out/q.json 2>$R/gpurun_out/q.err || exit 3
python3 -c "
import json; d=json.load(open('$R/gpurun_out/q.json')); i=d['initial_tick']; print({k:i[k] for k in ('wall_ms','kernel_ms','k_emit_ms','host_ms')}, d['ms_per_step'])"
