# C4 at several last-chunk cuts (KWOK_INGEST_LAST_CUT), the C4 probe's ms per step
set -o pipefail
R=$GRAFT_REPO_ROOT
for C in 0.4 0.6 0.75; do
  KWOK_INGEST_LAST_CUT=$C timeout -k 10 300 python -u $R/tools/c4_probe.py --ticks 8 > $R/gpurun_out/cut_$C.json 2> $R/gpurun_out/cut_$C.err || { tail -20 $R/gpurun_out/cut_$C.err; exit 1; }
  echo "cut $C: $(grep '^{' $R/gpurun_out/cut_$C.json | head -c 200)"
done
