set -o pipefail
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=3 KWOK_TICK_TRACE_SLOW=1 timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 3 > gpurun_out/s6_trace.json 2> gpurun_out/s6_trace.err || { tail -5 gpurun_out/s6_trace.err; exit 1; }
grep "kwok trace" gpurun_out/s6_trace.err | tail -60
timeout -k 10 600 python -u bench.py --leg emul --churn-ticks 3 > gpurun_out/s6_emul.json 2> gpurun_out/s6_emul.err || { tail -20 gpurun_out/s6_emul.err; exit 2; }
tail -c 1200 gpurun_out/s6_emul.json
