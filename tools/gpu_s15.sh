set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s15 -o run -- python3 $R/bench.py --leg hb_once --steps 10 --churn-ticks 1 --json-ticks 2 > $R/gpurun_out/s15_hb.json 2> $R/gpurun_out/s15_hb.err || exit 4
grep json $R/gpurun_out/prof_s15/run_kernel_stats.csv
python3 -c "import json; d=json.loads(open('$R/gpurun_out/s15_hb.json').read().strip().splitlines()[-1]); c=d['churn_json']; print(c['ms_per_step'], c['decode_ingest_ms'], c['documents_per_s'])"
