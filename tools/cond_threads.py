#!/usr/bin/env python3
"""bond_cond trials on K host threads, one context (and stream) each, on one
GPU: does a small-lattice ensemble gain from concurrent contexts?

  python tools/cond_threads.py [--L 64 --trials 8 --threads 1,2,4,8]
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=64)
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--threads", default="1,2,4,8")
    args = ap.parse_args()
    from percolation_amd import api
    L_ = args.L
    for K in map(int, args.threads.split(",")):
        ctxs = [api.Context(0, L_, L_, 0) for _ in range(K)]
        for c in ctxs:  # warm-up
            api.bond_cond_grid(0, L_, L_, 0, numtrials=1, itmax=10 ** 6, ctx=c, with_labels=False)
        res = [None] * K

        def work(k):
            tr = list(range(k, args.trials, K))
            res[k] = api.bond_cond_grid(0, L_, L_, 0, trials=tr, itmax=10 ** 6, ctx=ctxs[k],
                                        with_labels=False)
        t0 = time.perf_counter()
        th = [threading.Thread(target=work, args=(k,)) for k in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        npts = sum(len(t["rows"]) for r in res for t in r)
        print(json.dumps(dict(L=L_, threads=K, trials=args.trials, trials_per_s=round(args.trials / wall, 3),
                              points=npts, ms_per_point=round(wall * 1e3 / npts, 3))), flush=True)
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()
