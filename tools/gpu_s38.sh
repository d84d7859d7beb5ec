# the emulated-8-rank leg with its steady ticks also queued two deep (as the headline)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u bench.py --leg emul --churn-ticks 3 > gpurun_out/s38.json 2> gpurun_out/s38.err || { tail -20 gpurun_out/s38.err; exit 4; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print({k: d[k] for k in ('steady_ms_per_tick', 'steady_queued_ms_per_tick')}, d['steady_phase_ms']['kernel'], d['churn']['tick_ms'])" gpurun_out/s38.json
