#!/usr/bin/env python3
"""Time the CG kernels of one assembled L x L system under several
environment settings of libperc's research knobs (PERC_MARCH_NW,
PERC_MARCH_PACE, ...), a fresh context per setting (the knobs are read
when the lattice is built).  perc_bench_kernel 1 = P+S, 2 = B, 5 = one
whole iteration.

  python tools/env_probe.py --L 4096 --sets '[{}, {"PERC_MARCH_NW": "16"}]'
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
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--sets", required=True)
    ap.add_argument("--which", default="1,2,5")
    args = ap.parse_args()
    import torch
    from percolation_amd import api
    sets = json.loads(args.sets)
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    o = (np.random.default_rng(1234).permutation(nb)[:tb] + 1).astype(np.int32)
    dev_o = torch.from_numpy(o).cuda()
    N = L_ * L_ - 2 * L_
    out = {}
    for rnd in range(args.rounds):  # rounds interleave the settings (box drift)
        for env in sets:
            keys = set()
            for s_ in sets:
                keys |= set(s_)
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update({k: str(v) for k, v in env.items()})
            with api.Context(0, L_, L_, 0) as ctx:
                r = ctx.bondc_realisation(None, tb, tol=1e-8, itmax=20, device_ptr=dev_o.data_ptr())
                t = {w: ctx.bench_kernel(w, args.reps) for w in map(int, args.which.split(","))}
            name = json.dumps(env, sort_keys=True)
            row = dict(ps_ms=t.get(1), b_ms=t.get(2), iter_ms=t.get(5), nspan=r["nspan"])
            if t.get(5):
                row["iter_gbs"] = round(60 * N / t[5] / 1e6, 1)
            if t.get(4):
                row["copy_ms"] = t[4]
                row["copy_gbs"] = round(2 * 8 * (64 << 20) / t[4] / 1e6, 1)
            if t.get(1):
                row["ps_gbs"] = round(34 * N / t[1] / 1e6, 1)
            out.setdefault(name, []).append(row)
            print("round %d %s %s" % (rnd, name, json.dumps(row)), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
