set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_json_gpu.py tests/test_controller_gpu.py -k 'not 1m_10m' -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/json_t.log 2>&1 || { tail -20 $R/gpurun_out/json_t.log; exit 1; }
tail -2 $R/gpurun_out/json_t.log
KWOK_INGEST_PROF=1 timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --churn-ticks 2 --flap-ticks 0 --emulate-ranks 0 --c2 0 --json-ticks 3 > $R/gpurun_out/bench_json.json 2> $R/gpurun_out/bench_json.err || { tail -30 $R/gpurun_out/bench_json.err; exit 2; }
python3 -c "
import json; d=json.load(open('$R/gpurun_out/bench_json.json')); h=d['heartbeat_once']
c=h['churn_json']; print({k:c[k] for k in ('ms_per_step','decode_ingest_ms','tick_ms','documents_per_s')}, c['host_codec']['ms'])"
grep "kwok json" $R/gpurun_out/bench_json.err | tail -6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_json -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --churn-ticks 1 --flap-ticks 0 --emulate-ranks 0 --c2 0 --json-ticks 2 --roofline-ticks 0 > $R/gpurun_out/prof_json.log 2>&1 || exit 3
T=$(find $R/gpurun_out/prof_json -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 3 --out $R/gpurun_out/ktrace_json.txt | grep -E "json|ing_|k_tick|k_once|kernel"
