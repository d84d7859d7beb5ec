#!/bin/bash
# k_emit without the per-block spec-program / blob caches in LDS (32 KB per block:
# 5 blocks per CU instead of 4): emitter parity tests on the variant, then A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
V=$R/kwok_amd/lib/var/libkwok_engine_nocache.so
KWOK_ENGINE_LIB=$V timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_emit_paths_gpu.py tests/test_custom_template_gpu.py tests/test_parity_gpu.py > $R/gpurun_out/rag_tests.log 2>&1
rc=$?
tail -2 $R/gpurun_out/rag_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $R/gpurun_out/rag_tests.log | head -30; exit $rc; }
bash $R/tools/ab_emit.sh "nt4=-" "nc5=$V" "nt4b=-" "nc5b=$V" "nc4=$V:KWOK_EMIT_BLOCKS_PER_CU=4" || exit 1
python3 - <<'PY'
import json
for n in ['nt4','nc5']:
    d=json.load(open('/root/repo/gpurun_out/ab_%s.json'%n)); print(n, 'emit grid', d.get('config',{}).get('emit_grid'), 'initial wall', d['initial_tick']['wall_ms'], 'churn kernels', d['churn']['kernel_ms'])
PY
exit 0
