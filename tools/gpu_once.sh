#!/bin/bash
# k_once checkpoint: its GPU tests + the heartbeat-once parity / drop-in tests,
# then the heartbeat-once steady tick at 1M x 10M (tools/once_probe.py) with
# and without k_once, and a kernel trace.  Usage: gpu_once.sh TAG
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_once_gpu.py tests/test_cni_gpu.py tests/test_parity_gpu.py tests/test_controller_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > $R/gpurun_out/once_tests_$TAG.log 2>&1
rc=$?
tail -4 $R/gpurun_out/once_tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $R/gpurun_out/once_tests_$TAG.log | head -30; exit $rc; }
# (AB=KWOK_ONCE_SUM: per-bucket summaries on / off instead of k_once on / off)
AB=${AB:-KWOK_ONCE}
for ab in 1 0 1 0; do
  env $AB=$ab timeout -k 10 200 python tools/once_probe.py 200 "$AB=$ab" 2>&1 | tail -1 || exit 3
done
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=8 timeout -k 10 200 python tools/once_probe.py 40 trace > $R/gpurun_out/once_trace_$TAG.txt 2>&1 || exit 4
grep -E "kwok trace|queued" $R/gpurun_out/once_trace_$TAG.txt | head -30
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_once_$TAG -o run -- python3 $R/tools/once_probe.py 60 prof > $R/gpurun_out/once_prof_$TAG.log 2>&1 || exit 5
T=$(find $R/gpurun_out/prof_once_$TAG -name 'run_kernel_trace.csv' | head -n 1)
python3 $R/tools/trace_summary.py "$T" --last 100 --out $R/gpurun_out/ktrace_once_$TAG.txt || exit 6
cat $R/gpurun_out/ktrace_once_$TAG.txt | head -20
exit 0
