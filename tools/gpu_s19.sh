set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 1100 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/test_ingest_tick_gpu.py tests/test_c4_churn_gpu.py tests/test_parity_gpu.py tests/test_growth_gpu.py tests/test_emit_paths_gpu.py tests/test_once_gpu.py -k "not metric_size or ingest_then_tick" > gpurun_out/s19_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s19_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/s19_tests.log | head -20; exit 3; }
for v in two together two2 together2; do
  case $v in together*) F=--together;; *) F=;; esac
  KWOK_INGEST_PROF=0 timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 6 $F > gpurun_out/s19_$v.json 2> gpurun_out/s19_$v.err || { tail -5 gpurun_out/s19_$v.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'step %.3f (median %.3f) ingest %.3f tick %.3f kernel %.3f' % (d['ms_per_step'], d['median_ms']['step'], d['ingest_ms'], d['tick_ms'], d['kernel_ms']))" gpurun_out/s19_$v.json $v
done
