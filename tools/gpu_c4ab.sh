#!/bin/bash
# C4 churn A/B on the heartbeat-once engine and the full-body engine: each
# variant "NAME=ENV=V,ENV=V" runs tools/c4_probe.py --ticks 6 (once and full).
# Usage: gpu_c4ab.sh TAG NAME=ENVS ...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}; [ "$envs" = "$spec" ] && envs=""
  for mode in once full; do
    flag=""; [ $mode = once ] && flag="--once"
    env ${envs//,/ } timeout -k 10 300 python -u $R/tools/c4_probe.py $flag --ticks 6 > $R/gpurun_out/c4ab_${TAG}_${name}_$mode.json 2> $R/gpurun_out/c4ab_${TAG}_${name}_$mode.err || { echo "FAIL $name $mode"; tail -5 $R/gpurun_out/c4ab_${TAG}_${name}_$mode.err; exit 1; }
    echo "$name $mode $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('step %.3f tick %.3f kernel %.3f phases %s' % (d['median_ms']['step'], d['median_ms']['tick'], d['kernel_ms'], {k: round(v, 3) for k, v in d['phase_ms'].items() if v}))" $R/gpurun_out/c4ab_${TAG}_${name}_$mode.json)"
  done
done
