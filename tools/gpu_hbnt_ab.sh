# steady tick with the heartbeat stream non-temporal (default for streams > 256 MB) or plain (KWOK_HB_NT)
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in 1 0 1 0; do
  KWOK_HB_NT=$v timeout -k 10 200 python3 $R/bench.py --steps 300 --warmup 5 --cpu-baseline 0 --churn-ticks 0 --flap-ticks 0 --once-ticks 0 --emulate-ranks 0 --c2 0 --json-ticks 0 --roofline-ticks 20 > $R/gpurun_out/hbnt_$v.json 2>/dev/null || { echo FAIL; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$R/gpurun_out/hbnt_$v.json').read().strip().splitlines()[-1]); print('nt=$v', round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5))"
done
