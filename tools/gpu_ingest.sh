# the ingest-touching GPU tests, then the C4 probe (tools/gpu_c4.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_c4_churn_gpu.py tests/test_ingest_chunks_gpu.py tests/test_growth_gpu.py tests/test_node_dir_gpu.py tests/test_c5_flap_gpu.py tests/test_json_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/ingest_t_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/ingest_t_$TAG.log; exit 1; }
tail -2 $R/gpurun_out/ingest_t_$TAG.log
bash $R/tools/gpu_c4.sh $TAG
