#!/bin/bash
# Fused k_pod_jobs at 4 waves per SIMD (launch bounds; a few spilled registers)
# against 3: the initial tick, alternating, one box.  Variant library built by
# tools/build_variant.sh w4 "" <source with FUSE ? 4>.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for V in "" w4 "" w4 "" w4; do
  L=""; [ -n "$V" ] && L=$R/kwok_amd/lib/var/libkwok_engine_$V.so
  KWOK_ENGINE_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --churn-ticks 0 > $R/gpurun_out/r6g_$V.json 2> $R/gpurun_out/r6g_$V.err || { tail -5 $R/gpurun_out/r6g_$V.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); i=d['initial_tick']; print('variant', sys.argv[2], 'init wall %.3f kernels %.3f emission %.3f' % (i['wall_ms'], i['kernel_ms'], i['emission_ms']))" $R/gpurun_out/r6g_$V.json "w3$V"
done
