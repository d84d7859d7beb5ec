#!/bin/bash
# bench + kernel-trace profile (round 1)
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/bench_r1a.json 2> gpurun_out/bench_r1a.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r1a -o run -- python3 $R/bench.py --steps 50 --warmup 3 --cpu-baseline 0 > $R/gpurun_out/bench_r1a_prof.json 2>&1
rc=$?
cat $R/gpurun_out/bench_r1a.json
exit $rc
