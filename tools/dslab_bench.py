#!/usr/bin/env python3
"""One L x L conductance solve split over the processes of a torchrun job
(percolation_amd/dslab.py), against the single-process solves on rank 0.
Prints one JSON line: ms per iteration of the split solve and of the
single-process slab solve (perc_set_slabs(1) path: one process, launched
kernels) -- the cost of the host-driven exchange.

  torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/dslab_bench.py [--L 4096]
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
    ap.add_argument("--tol", type=float, default=1e-8)
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    from percolation_amd import _lib as PL
    from percolation_amd import api, dslab
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    o = (np.random.default_rng(1234).permutation(nb)[:tb] + 1).astype(np.int32)
    out = {}
    with api.Context(0, L_, L_, 0, device=local) as ctx:
        ctx.occupy(PL.BOND, bond_order=o, nbonds_=tb)
        ctx.label()
        dist.barrier()
        t0 = time.perf_counter()
        r = dslab.conductance(ctx, tol=args.tol, itmax=10 ** 6)
        torch.cuda.synchronize()
        dist.barrier()
        t = time.perf_counter() - t0
        out["split"] = dict(processes=world, iter=r["iter"], gtop=r["gtop"],
                            ms_per_iteration=round(t * 1e3 / max(r["iter"], 1), 5))
        if rank == 0:
            for mode, name in ((PL.MARCH_ALT, "one_process_rowmajor_q_stored"),
                               (PL.MARCH_DEFAULT, "one_process_default")):
                ctx.set_march_mode(mode)
                t0 = time.perf_counter()
                c = ctx.conductance(tol=args.tol, itmax=10 ** 6)
                t = time.perf_counter() - t0
                out[name] = dict(iter=c["iter"], gtop=c["gtop"],
                                 ms_per_iteration=round(t * 1e3 / max(c["iter"], 1), 5))
    if rank == 0:
        print(json.dumps(dict(L=L_, p=args.p, **out)), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
