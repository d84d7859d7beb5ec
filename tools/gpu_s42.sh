# k_ing_apply's check for a slot named twice in a chunk by LDS tags (a few ballot
# rounds instead of 63 lane reads): the ingest parity tests, then the C4 A/B against
# the previous build (prev) and the apply kernel's trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ingest_chunks_gpu.py tests/test_ingest_tick_gpu.py \
  tests/test_c4_churn_gpu.py tests/test_growth_gpu.py tests/test_parity_gpu.py tests/test_node_dir_gpu.py tests/test_use_checks_gpu.py > gpurun_out/s42_tests.txt 2>&1 || { tail -30 gpurun_out/s42_tests.txt; exit 3; }
tail -1 gpurun_out/s42_tests.txt
C4ARGS="--together --once" bash $R/tools/gpu_c4_ab.sh prev=$R/kwok_amd/lib/var/libkwok_engine_prev.so new=- prev2=$R/kwok_amd/lib/var/libkwok_engine_prev.so new2=- > /dev/null || exit 4
for v in prev new prev2 new2; do python3 -c "
import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'step %.3f ingest %.3f tick %.3f med %.3f' % (d['ms_per_step'], d['ingest_ms'], d['tick_ms'], d['median_ms']['step']))" $R/gpurun_out/c4ab_$v.json $v; done
cd /tmp && export TMPDIR=/tmp
for v in prev new; do
  L=$R/kwok_amd/lib/libkwok_engine.so; [ $v = prev ] && L=$R/kwok_amd/lib/var/libkwok_engine_prev.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s42_$v -o run -- python3 $R/tools/c4_probe.py --ticks 3 --once > $R/gpurun_out/prof_s42_$v.log 2>&1 || exit 5
  T=$(find $R/gpurun_out/prof_s42_$v -name 'run_kernel_trace.csv' | head -n 1)
  python3 $R/tools/trace_summary.py "$T" --last 6 --out $R/gpurun_out/ktrace_s42_$v.txt
  echo "== $v $(grep -E 'k_ing_apply' $R/gpurun_out/ktrace_s42_$v.txt)"
done
