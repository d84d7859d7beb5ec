set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && KWOK_INGEST_PROF=1 timeout -k 10 300 python -u tools/c4_probe.py --once --ticks 4 > gpurun_out/s17_c4.json 2> gpurun_out/s17_c4.err || { tail -5 gpurun_out/s17_c4.err; exit 4; }
grep "kwok" gpurun_out/s17_c4.err | tail -24
