set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_metric_gpu.py tests/test_emit_paths_gpu.py tests/test_c3_8rank_gpu.py tests/test_dist_gpu.py tests/test_use_checks_gpu.py > gpurun_out/s18_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s18_tests.log; [ $rc -eq 0 ] || exit 3
for v in fresh nofresh fresh2 nofresh2; do
  case $v in nofresh*) L=kwok_amd/lib/var/libkwok_engine_nofresh.so;; *) L=;; esac
  KWOK_ENGINE_LIB=$L timeout -k 10 300 python -u bench.py --leg hb_once --steps 10 --churn-ticks 0 --json-ticks 0 > gpurun_out/s18_$v.json 2> gpurun_out/s18_$v.err || { tail -5 gpurun_out/s18_$v.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); i=d['initial_tick']; print(sys.argv[2], 'wall %.3f kernel %.3f emission %.3f' % (i['wall_ms'], i['kernel_ms'], i['emission_ms']))" gpurun_out/s18_$v.json $v
done
