# the pool-touching GPU tests, then the emulated-ranks leg (tools/emul_probe.py)
# plain and under a kernel trace: per-kernel stats and the timeline of the last
# churn tick
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_rccl_gpu.py tests/test_dist_gpu.py tests/test_c3_8rank_gpu.py tests/test_c4_churn_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/emul_t_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/emul_t_$TAG.log; exit 1; }
tail -2 $R/gpurun_out/emul_t_$TAG.log
timeout -k 10 300 python -u $R/tools/emul_probe.py > $R/gpurun_out/emul_$TAG.json 2> $R/gpurun_out/emul_$TAG.err || { tail -20 $R/gpurun_out/emul_$TAG.err; exit 1; }
python3 $R/tools/last_json.py $R/gpurun_out/emul_$TAG.json steady_ms_per_tick churn
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_emul_$TAG -o run -- python3 $R/tools/emul_probe.py --churn-ticks 2 > $R/gpurun_out/prof_emul_$TAG.log 2>&1 || exit 3
T=$(find $R/gpurun_out/prof_emul_$TAG -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 3 --out $R/gpurun_out/ktrace_emul_$TAG.txt
python3 $R/tools/timeline.py "$T" --last 20 > $R/gpurun_out/timeline_emul_$TAG.txt
cat $R/gpurun_out/timeline_emul_$TAG.txt
