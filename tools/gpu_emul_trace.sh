# the emulated-ranks leg with per-block stamps (KWOK_TICK_TRACE; the churn ticks only)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
KWOK_TICK_TRACE=1 KWOK_TICK_TRACE_SKIP=24 timeout -k 10 300 python -u $R/tools/emul_probe.py > $R/gpurun_out/emul_tr_$TAG.json 2> $R/gpurun_out/emul_tr_$TAG.err || { tail -20 $R/gpurun_out/emul_tr_$TAG.err; exit 1; }
grep "kwok trace" $R/gpurun_out/emul_tr_$TAG.err
