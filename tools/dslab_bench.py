#!/usr/bin/env python3
"""Per-iteration cost of the split solve's exchange at K = 1 (one GPU):
the single-context solve with the slab kernels' march (MARCH_ALT, q stored)
against perc_dslab_solve_group over RCCL and through the host, the loop
inside libperc (and, with --torch, percolation_amd/dslab.py's Python loop
over a torch.distributed "nccl" group of one).  Fixed iteration counts
(tol 0): ms per iteration = the slope between a solve of `iters` and one of
iters / 2 iterations (set-up, communicator creation and currents cancel).

  python tools/dslab_bench.py --L 4096 --iters 2000
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--torch", action="store_true")
    args = ap.parse_args()
    from percolation_amd import _lib as PL
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    seed = int(api.trial_seeds(58302, 1)[0])
    out = dict(L=L_, p=args.p, iterations=args.iters)

    def ctx_new():
        c = api.Context(0, L_, L_, 0)
        c.set_march_mode(PL.MARCH_ALT)
        c.occupy_random(PL.BOND, 0, tb, seed)
        c.label()
        return c

    def slope(fn):
        fn(50)  # warm
        res = []
        for n in (args.iters // 2, args.iters):
            t = time.perf_counter()
            it = fn(n - 1)
            res.append((time.perf_counter() - t, it))
        (t1, i1), (t2, i2) = res
        return round((t2 - t1) * 1e3 / (i2 - i1), 5)

    c = ctx_new()
    out["single_context_ms_per_it"] = slope(lambda n: c.conductance(tol=0.0, itmax=n)["iter"])
    c.close()
    for name, xp in (("group_rccl", PL.XPORT_RCCL), ("group_host", PL.XPORT_HOST)):
        c = ctx_new()
        out[name + "_ms_per_it"] = slope(
            lambda n: api.dslab_solve_group([c], xport=xp, tol=0.0, itmax=n)["iter"])
        c.close()
    if args.torch:
        import torch
        import torch.distributed as dist
        from percolation_amd import dslab
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        c = ctx_new()
        out["python_dslab_nccl_ms_per_it"] = slope(lambda n: dslab.conductance(c, tol=0.0, itmax=n)["iter"])
        c.close()
        dist.destroy_process_group()
    for k in ("group_rccl", "group_host", "python_dslab_nccl"):
        if k + "_ms_per_it" in out:
            out[k + "_overhead_us"] = round((out[k + "_ms_per_it"] - out["single_context_ms_per_it"]) * 1e3, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
