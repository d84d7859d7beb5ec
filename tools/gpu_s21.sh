set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in zc copy zc2 copy2; do
  case $v in copy*) E="KWOK_INGEST_ZC=0";; *) E="KWOK_NOTHING=1";; esac
  env $E timeout -k 10 300 python -u bench.py --leg flap_once --flap-ticks 8 > gpurun_out/s21_$v.json 2> gpurun_out/s21_$v.err || { tail -5 gpurun_out/s21_$v.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f json %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['from_json']['ms_per_step']))" gpurun_out/s21_$v.json "$v $E"
done
