#!/usr/bin/env python3
"""Probe the register-march loop variants (perc_set_march_mode) and band
heights on one realisation: per-kernel and whole-iteration times
(perc_bench_kernel 1, 2, 5), then full solves per mode.

  python tools/march_probe.py [--L 4096 --p 0.6 --solve-L 1024]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--solve-L", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--rows", default="0")
    ap.add_argument("--modes", default="2,0,6,4,7,5")
    ap.add_argument("--solve-modes", default="2,6,7,2")
    args = ap.parse_args()
    import torch
    import percolation_amd as P
    from percolation_amd import api
    out = {}
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    o = (np.random.default_rng(1234).permutation(nb)[:tb] + 1).astype(np.int32)
    dev_o = torch.from_numpy(o).cuda()
    N = L_ * L_ - 2 * L_
    with api.Context(0, L_, L_, 0) as ctx:
        r = ctx.bondc_realisation(None, tb, tol=1e-8, itmax=20, device_ptr=dev_o.data_ptr())
        print("assembled L=%d: nspan=%d" % (L_, r["nspan"]), file=sys.stderr, flush=True)
        for rows in [int(x) for x in args.rows.split(",")]:
            ctx.set_march_rows(rows)
            for mode in [int(x) for x in args.modes.split(",")]:
                ctx.set_march_mode(mode)
                t = {w: ctx.bench_kernel(w, args.reps) for w in (5, 1, 2, 5)}
                key = "rows%d_mode%d" % (rows, mode)
                out[key] = dict(iter_ms=t[5], ps_ms=t[1], b_ms=t[2],
                                iter_gbs=(52 if mode & 1 else 60) * N / t[5] / 1e6)
                print(key, json.dumps(out[key]), file=sys.stderr, flush=True)
        ctx.set_march_rows(0)
        ctx.set_march_mode(P.MARCH_DEFAULT)
    L_ = args.solve_L
    if L_ <= 0:
        print(json.dumps(out))
        return
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    o = (np.random.default_rng(99).permutation(nb)[:tb] + 1).astype(np.int32)
    dev_o = torch.from_numpy(o).cuda()
    with api.Context(0, L_, L_, 0) as ctx:
        for mode in [int(x) for x in args.solve_modes.split(",")]:
            ctx.set_march_mode(mode)
            r = ctx.bondc_realisation(None, tb, tol=1e-8, itmax=10 ** 6,
                                      device_ptr=dev_o.data_ptr())
            key = "solve%d_mode%d" % (L_, mode)
            out[key] = dict(iter=r["iter"], gtop=r["gtop"], gbot=r["gbot"],
                            ms=r["t_solve_ms"], ms_per_iter=r["t_solve_ms"] / max(r["iter"], 1))
            print(key, json.dumps(out[key]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
