#!/usr/bin/env python3
"""Throughput of the §8(f) callers around the hot path on one GPU:

  bond_perc / site_perc (threshold scans, Square/bond_perc.f:86-369,
    site_perc.f:69-260): per trial the reference shuffle (host), the first
    spanning occupation count by GPU bisection (perc_first_spanning, ~log2 N
    labelings), the largest and spanning cluster sizes at that count
    (perc_cluster_sizes, GPU);
  bond_cond (Square/bond_cond.f:123-498): per trial one labeling +
    conductance solve at each of the ~100 grid points, then the pc scan.

Prints one JSON line per workload: trials/s and the per-trial split.

  python tools/scan_bench.py [--L 256,1024 --trials 8 --cond-L 64,256 --cond-trials 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def scan(api, L_mod, lat, L_, kind, trials):
    N = api.nbonds(lat, L_, L_, 0) if kind == L_mod.BOND else L_ * L_
    seeds = api.trial_seeds(58302, trials, scale=1000000)
    t_shuf = t_gpu = t_rep = 0.0
    firsts = []
    with api.Context(lat, L_, L_, 0) as ctx:
        api.first_spanning(ctx, api.shuffled_ids(N, 12345), kind, N)  # warm-up
        t0 = time.perf_counter()
        for ii in range(trials):
            a = time.perf_counter()
            order = api.shuffled_ids(N, int(seeds[ii]))
            b = time.perf_counter()
            first = api.first_spanning(ctx, order, kind, N)
            c = time.perf_counter()
            ctx.cluster_sizes()  # maxcs, spanning size on the GPU (perc_cluster_sizes)
            d = time.perf_counter()
            t_shuf += b - a
            t_gpu += c - b
            t_rep += d - c
            firsts.append(first)
        wall = time.perf_counter() - t0
    return dict(workload="%s_perc %s L=%d" % ("bond" if kind == L_mod.BOND else "site",
                                               "square" if lat == 0 else "triangular", L_),
                trials=trials, trials_per_s=round(trials / wall, 3),
                ms_per_trial=round(wall * 1e3 / trials, 2),
                host_shuffle_ms=round(t_shuf * 1e3 / trials, 2),
                gpu_first_spanning_ms=round(t_gpu * 1e3 / trials, 2),
                gpu_cluster_sizes_ms=round(t_rep * 1e3 / trials, 2),
                mean_first_fraction=round(float(np.mean(firsts)) / N, 5))


def cond(api, lat, L_, trials):
    with api.Context(lat, L_, L_, 0) as ctx:
        api.bond_cond_grid(lat, L_, L_, 0, numtrials=1, itmax=10 ** 6, ctx=ctx)  # warm-up
        t0 = time.perf_counter()
        out = api.bond_cond_grid(lat, L_, L_, 0, numtrials=trials, itmax=10 ** 6, ctx=ctx)
        wall = time.perf_counter() - t0
    npts = sum(len(t["rows"]) for t in out)
    iters = sum(r["iter"] for t in out for r in t["rows"])
    return dict(workload="bond_cond %s L=%d" % ("square" if lat == 0 else "triangular", L_),
                trials=trials, trials_per_s=round(trials / wall, 4),
                ms_per_trial=round(wall * 1e3 / trials, 1), grid_points=npts,
                points_per_s=round(npts / wall, 2), cg_iterations=iters,
                ms_per_point=round(wall * 1e3 / max(npts, 1), 3))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", default="256,1024")
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--cond-L", default="64,256")
    ap.add_argument("--cond-trials", type=int, default=2)
    args = ap.parse_args()
    from percolation_amd import _lib as L_mod
    from percolation_amd import api
    for L_ in map(int, args.L.split(",")):
        for kind in (L_mod.BOND, L_mod.SITE):
            print(json.dumps(scan(api, L_mod, 0, L_, kind, args.trials)), flush=True)
    for L_ in map(int, args.cond_L.split(",")):
        print(json.dumps(cond(api, 0, L_, args.cond_trials)), flush=True)


if __name__ == "__main__":
    main()
