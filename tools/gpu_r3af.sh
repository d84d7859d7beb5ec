#!/bin/bash
# k_emit store flavour x blocks per CU (the 7.2 GB fill: plain stores at few waves
# per CU 5.78 TB/s, non-temporal 5.36 TB/s): initial-tick / churn k_emit A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
P=$R/kwok_amd/lib/var/libkwok_engine_plain.so
bash $R/tools/ab_emit.sh "nt4=-" "nt2=-:KWOK_EMIT_BLOCKS_PER_CU=2" "nt1=-:KWOK_EMIT_BLOCKS_PER_CU=1" \
  "pl4=$P" "pl2=$P:KWOK_EMIT_BLOCKS_PER_CU=2" "pl1=$P:KWOK_EMIT_BLOCKS_PER_CU=1" "nt4b=-" "pl2b=$P:KWOK_EMIT_BLOCKS_PER_CU=2" || exit 1
exit 0
