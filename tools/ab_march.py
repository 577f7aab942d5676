#!/usr/bin/env python3
"""Same-box A/B of march variants (environment knobs read at context
creation) on one L x L bond realisation: iterations, Gtop/Gbot (must be
bitwise equal across variants that keep the reduction order), P / B
average launch times (kernel dispatch timestamps, 1 iteration in 8) and
the solve's wall time.  Variants run interleaved, each `--rounds` times.

  python tools/ab_march.py --L 4096 --variants "DEFER=0,SAUX=2;DEFER=1,SAUX=2"
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
    ap.add_argument("--ii", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--tol", type=float, default=1e-8)
    ap.add_argument("--itmax", type=int, default=60000)
    ap.add_argument("--variants", default="DEFER=0;DEFER=1")
    args = ap.parse_args()
    import percolation_amd as P
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    seed = int(api.trial_seeds(58302, args.ii)[args.ii - 1])
    variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in args.variants.split(";")]
    res = {}
    for rnd in range(args.rounds):
        for v in variants:
            key = ",".join("%s=%s" % kv for kv in sorted(v.items())) or "default"
            for k_, val in v.items():
                os.environ["PERC_MARCH_" + k_] = val
            with api.Context(0, L_, L_, 0) as ctx:
                ctx.occupy_random(P._lib.BOND, 0, tb, seed)
                li = ctx.label()
                assert li["nspan"] > 0
                ctx.set_kernel_timing(True)
                ctx.kernel_stats(reset=True)
                t0 = time.perf_counter()
                c = ctx.conductance(tol=args.tol, itmax=args.itmax)
                wall = time.perf_counter() - t0
                ks = ctx.kernel_stats(reset=True)
            for k_ in v:
                del os.environ["PERC_MARCH_" + k_]
            row = dict(variant=key, round=rnd, iter=c["iter"], gtop=c["gtop"].hex(),
                       gbot=c["gbot"].hex(), wall_s=round(wall, 4),
                       ms_per_iter=round(wall * 1e3 / c["iter"], 5),
                       p_ms=round(ks["spmv_ms"] / max(ks["spmv_n"], 1), 5),
                       b_ms=round(ks["resid_ms"] / max(ks["resid_n"], 1), 5))
            print(json.dumps(row), flush=True)
            res.setdefault(key, []).append(row)
    base = None
    for key, rows in res.items():
        g = {(r["iter"], r["gtop"], r["gbot"]) for r in rows}
        if base is None:
            base = g
        print("%-30s iter/G %s  ms/it %s  P %s  B %s  %s" % (
            key, "same" if g == base else "DIFF", [r["ms_per_iter"] for r in rows],
            [r["p_ms"] for r in rows], [r["b_ms"] for r in rows], sorted(g)[0][0]), flush=True)


if __name__ == "__main__":
    main()
