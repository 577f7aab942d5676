#!/usr/bin/env python3
"""bond_cond trials per second on one GPU through perc_ensemble_bond_cond
with W workers (contexts, host threads, streams) per device.

  python tools/cond_workers.py [--L 64,128 --trials 16 --workers 1,2,4,8,16]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", default="64,128")
    ap.add_argument("--trials", type=int, default=16)
    ap.add_argument("--workers", default="1,2,4,8,16")
    args = ap.parse_args()
    from percolation_amd import api
    for L_ in map(int, args.L.split(",")):
        for W in map(int, args.workers.split(",")):
            with api.Ensemble(0, L_, L_, 0, ndev=1, workers=W) as e:
                e.bond_cond(58302, min(W, args.trials))  # warm-up: every context once
                t0 = time.perf_counter()
                res, stats = e.bond_cond(58302, args.trials)
                wall = time.perf_counter() - t0
            npts = sum(len(t["rows"]) for t in res)
            print(json.dumps(dict(workload="bond_cond square L=%d (perc_ensemble, 1 GPU)" % L_,
                                  workers=W, trials=args.trials,
                                  trials_per_s=round(args.trials / wall, 3), points=npts,
                                  ms_per_point=round(wall * 1e3 / npts, 3))), flush=True)


if __name__ == "__main__":
    main()
