set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s13 -o run -- python3 $R/tools/emul_probe.py --churn-ticks 2 > $R/gpurun_out/s13_emul.json 2> $R/gpurun_out/s13_emul.err || exit 5
T=$(find $R/gpurun_out/prof_s13 -name run_kernel_trace.csv); python3 $R/tools/timeline.py $T --last 60 > $R/gpurun_out/s13_timeline.txt
cd $R && KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=4 timeout -k 10 300 python -u tools/emul_probe.py --churn-ticks 0 > gpurun_out/s13_tr.json 2> gpurun_out/s13_tr.err || { tail -20 gpurun_out/s13_tr.err; exit 6; }
grep "kwok trace" gpurun_out/s13_tr.err | tail -40
