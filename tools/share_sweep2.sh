#!/bin/bash
R=$GRAFT_REPO_ROOT
source <(sed -n '/^run()/,/^}/p' $R/tools/share_sweep.sh)
for rep in 1 2; do
for s in 921 880 860 840 820; do run KWOK_TICK_STREAM_SHARE=$s; done
run KWOK_TICK_STREAMERS_PER_CU=2 KWOK_TICK_STREAM_SHARE=860
run KWOK_TICK_STREAMERS_PER_CU=2 KWOK_TICK_STREAM_SHARE=900
done
