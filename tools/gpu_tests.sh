# the whole GPU suite (stops at the first failure)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/tests_$TAG.log 2>&1 || { tail -40 $R/gpurun_out/tests_$TAG.log; exit 1; }
tail -3 $R/gpurun_out/tests_$TAG.log
