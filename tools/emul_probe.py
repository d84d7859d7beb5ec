"""The bench's emulated-ranks leg alone (KWOK_FORCE_MULTI + KWOK_EMULATE_RANKS):
one rank's 1M x 10M fleet whose BACK folds `ranks` ranks' messages and lists;
prints the leg's JSON (steady and churn ticks).  tools/gpu_emul.sh runs it under
a kernel trace to split the churn tick's N-dependent pool work by kernel.

usage: emul_probe.py [--ranks 8] [--churn-ticks 3]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--churn-ticks", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    a = ap.parse_args()
    print(json.dumps(bench.emulated_ranks_leg(a.nodes, a.ranks, 10, a.churn_ticks)), flush=True)


if __name__ == "__main__":
    main()
