set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && KWOK_INGEST_PROF=1 timeout -k 10 300 python -u bench.py --leg flap_once --flap-ticks 3 > gpurun_out/s16_flap.json 2> gpurun_out/s16_flap.err || { tail -5 gpurun_out/s16_flap.err; exit 4; }
grep "kwok" gpurun_out/s16_flap.err | tail -30
