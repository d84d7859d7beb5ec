set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in base cut3 cut5 ch3 base2 cut3b; do
  case $v in cut3*) E="KWOK_INGEST_LAST_CUT=0.3";; cut5) E="KWOK_INGEST_LAST_CUT=0.5";; ch3) E="KWOK_INGEST_CHUNK=700000";; *) E="KWOK_NOTHING=1";; esac
  env $E timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 6 --together > gpurun_out/s20_$v.json 2> gpurun_out/s20_$v.err || { tail -5 gpurun_out/s20_$v.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step %.3f (median %.3f) ingest %.3f tick %.3f' % (d['ms_per_step'], d['median_ms']['step'], d['ingest_ms'], d['tick_ms']))" gpurun_out/s20_$v.json "$v $E"
done
