#!/usr/bin/env python3
"""Labeling-side timing probe: per realisation, device-drawn
bond occupancy (perc_occupy_random) + labeling + spanning test
(perc_label) + Kirchhoff assembly (perc_conductance with itmax 1, whose
t_assemble_ms is the assembly alone).  Wall times per phase after a
synchronize; run under `rocprofv3 --kernel-trace --stats` for per-kernel
times.

  python tools/label_probe.py [--L 4096 --p 0.6 --reps 8]
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
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    import torch
    from percolation_amd import api
    from percolation_amd import _lib as PL
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    rows = []
    with api.Context(0, L_, L_, 0) as ctx:
        for k in range(args.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.occupy_random(PL.BOND, 0, tb, 1000 + k)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            li = ctx.label()
            t2 = time.perf_counter()
            c = ctx.conductance(tol=1e-8, itmax=1) if li["nspan"] else {"t_assemble_ms": 0.0}
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            if k:
                rows.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, c["t_assemble_ms"], (t3 - t2) * 1e3,
                             li["nspan"]))
    med = lambda j: sorted(r[j] for r in rows)[len(rows) // 2]
    print(json.dumps(dict(L=L_, p=args.p, reps=args.reps, occupy_ms=round(med(0), 4),
                          label_ms=round(med(1), 4), assemble_ms=round(med(2), 4),
                          cond_itmax1_ms=round(med(3), 4),
                          nspan=[r[4] for r in rows])))


if __name__ == "__main__":
    main()
