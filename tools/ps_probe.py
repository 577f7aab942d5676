"""Kernel A/B probe: one bond realisation per lattice size (uniform order,
seed tseed(1)) solved in full -- its (iter, Gtop, Gbot, err) is the bitwise
fingerprint a kernel variant must reproduce -- then k_cg_ps / k_cg_b timed
in isolation on the assembled L=4096 system (perc_bench_kernel 1 / 2).
Kernel variants are picked by environment switches read in libperc.
Usage: python tools/ps_probe.py [--sizes 1024 4096] [--reps 300]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from percolation_amd import api  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[1024, 4096])
    ap.add_argument("--p", type=float, default=0.60)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--tag", default=os.environ.get("PERC_PS_VARIANT", "0"))
    ap.add_argument("--march-rows", type=int, default=int(os.environ.get("PERC_MARCH_ROWS", "0")),
                    help="band height of the register-march kernel (0: auto)")
    ap.add_argument("--itmax", type=int, default=10**6,
                    help="small values: timing only (no fingerprint), for variants that "
                         "do not compute the real iteration")
    a = ap.parse_args()
    seed = int(api.trial_seeds(58302, 1)[0])
    out = {"tag": a.tag}
    for L_ in a.sizes:
        nb = api.nbonds(0, L_, L_, 0)
        tb = int(a.p * nb)
        order = (np.random.default_rng(seed).permutation(nb)[:tb] + 1).astype(np.int32)
        with api.Context(0, L_, L_, 0) as ctx:
            ctx.set_march_rows(a.march_rows)
            if os.environ.get("PERC_MODE"):
                ctx.set_march_mode(int(os.environ["PERC_MODE"]))
            t0 = time.perf_counter()
            r = ctx.bondc_realisation(order, tb, tol=1e-8, itmax=a.itmax)
            t1 = time.perf_counter()
            d = {"iter": r["iter"], "gtop": r["gtop"].hex(), "gbot": r["gbot"].hex(),
                 "err": r["err"].hex() if "err" in r else None, "solve_s": round(t1 - t0, 3)}
            if r["perccln"]:
                N = ctx.N
                ps = ctx.bench_kernel(1, a.reps)
                b = ctx.bench_kernel(2, a.reps)
                d.update(ps_ms=round(ps, 5), b_ms=round(b, 5),
                         ps_gbs=round((34 * N + 32 * L_) / ps / 1e6, 1),
                         b_gbs=round(26 * N / b / 1e6, 1))
            out[L_] = d
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
