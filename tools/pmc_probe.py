#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes (tools/pmc_r2.sh): one assembled
L x L system, then a fixed dispatch set that every pass sees identically --
`--reps` whole CG iterations (perc_bench_kernel 5: the march P+S kernel then
the streaming B kernel, every launch doing work) and `--copies` STREAM
copies of 512 MB (perc_bench_kernel 4, a known byte count: the counter
calibration).  tools/pmc_reconcile.py reads the last `--reps` / `--copies`
dispatches of each kernel from every pass.

  python tools/pmc_probe.py [--L 4096 --p 0.6 --reps 64 --copies 16]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--reps", type=int, default=64)
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--march-mode", type=int, default=-1, help="perc_set_march_mode bits; -1: default")
    ap.add_argument("--kind", default="bond", choices=("bond", "sitebond"),
                    help="sitebond: a mixed occupation (--ps, --p) under ConductCalc's mixed rule")
    ap.add_argument("--ps", type=float, default=0.85)
    args = ap.parse_args()
    import torch
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    o = (np.random.default_rng(1234).permutation(nb)[:tb] + 1).astype(np.int32)
    dev_o = torch.from_numpy(o).cuda()
    with api.Context(0, L_, L_, 0) as ctx:
        if args.march_mode >= 0:
            ctx.set_march_mode(args.march_mode)
        if args.kind == "bond":
            r = ctx.bondc_realisation(None, tb, tol=1e-8, itmax=20, device_ptr=dev_o.data_ptr())
        else:  # the config-5 companion's matrix
            from percolation_amd import _lib as PL
            ctx.occupy_random(PL.SITEBOND, int(args.ps * L_ * L_), tb, 1234)
            r = ctx.label()
            ctx.conductance(PL.RULE_MIXED, PL.CUR_MATLAB, tol=1e-8, itmax=20)
        it_ms = ctx.bench_kernel(5, args.reps)
        cp_ms = ctx.bench_kernel(4, args.copies)
    # bench_kernel adds 3 untimed warmup launches per call
    print("nspan=%d iteration %.5f ms copy %.5f ms (dispatches: %d iterations, %d copies)"
          % (r["nspan"], it_ms, cp_ms, args.reps + 3, args.copies + 3), file=sys.stderr)


if __name__ == "__main__":
    main()
