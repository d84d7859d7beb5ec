set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_c4_churn_gpu.py tests/test_once_gpu.py tests/test_emit_paths_gpu.py tests/test_c5_flap_gpu.py -k "not metric_size or drop_in" > gpurun_out/s12_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s12_tests.log; [ $rc -eq 0 ] || exit 3
bash tools/gpu_c4ab.sh s12 intick= kernel=KWOK_SPARSE_JOBS=1 intick2= kernel2=KWOK_SPARSE_JOBS=1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s12 -o run -- python3 $R/tools/c4_probe.py --once --ticks 4 > $R/gpurun_out/s12_prof.json 2> $R/gpurun_out/s12_prof.err || exit 5
T=$(find $R/gpurun_out/prof_s12 -name run_kernel_trace.csv); python3 $R/tools/timeline.py $T --last 12
