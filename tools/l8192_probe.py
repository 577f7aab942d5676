#!/usr/bin/env python3
"""The march past the Infinity Cache (L = 8192): the row-major q-free march
(P on one round of slot-mapped bands, B on 8-row bands with nontemporal r(k)
loads), best of 3 x `reps` launches of perc_bench_kernel 1 (P), 2 (B) and 5
(a whole iteration), plus ms per iteration of fixed-iteration solves (the
slope between itmax/2 and itmax, tol 0); GB/s on 26 B/row for P and B.
(Round 4 also ran the strip-major march with nibble codes here: 0.734 vs
0.652 ms per iteration, profiles/r4_4_l8192_strips_ab.json; removed.)

  python tools/l8192_probe.py --L 8192 --reps 10
  python tools/l8192_probe.py --kind sitebond --ps 0.85 --p 0.85   # the config-5 companion
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
    ap.add_argument("--L", type=int, default=8192)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--kind", default="bond", choices=("bond", "sitebond"))
    ap.add_argument("--ps", type=float, default=0.85)
    ap.add_argument("--seed", type=int, default=777)
    args = ap.parse_args()
    from percolation_amd import _lib as PL
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    modes = {"rowmajor": PL.MARCH_DEFAULT}
    out = dict(L=L_)
    with api.Context(0, L_, L_, 0) as ctx:
        if args.kind == "bond":
            ctx.occupy_random(PL.BOND, 0, int(args.p * nb), args.seed)
            rule = (PL.RULE_BOND, PL.CUR_FORTRAN)
        else:  # ConductCalc's mixed rule (MATLAB/ConductCalc.m:136-165)
            ctx.occupy_random(PL.SITEBOND, int(args.ps * L_ * L_), int(args.p * nb), args.seed)
            rule = (PL.RULE_MIXED, PL.CUR_MATLAB)
        assert ctx.label()["nspan"] > 0
        N, _ = ctx.system_size()
        best = {(m, w): 9e9 for m in modes for w in (1, 2, 5)}
        info = {}
        for _ in range(3):
            for name, mode in modes.items():
                ctx.set_march_mode(mode)
                ctx.conductance(*rule, tol=1e-8, itmax=2)
                info[name] = ctx.march_info()
                for w in (1, 2, 5):
                    best[(name, w)] = min(best[(name, w)], ctx.bench_kernel(w, args.reps))
        for name, mode in modes.items():
            ctx.set_march_mode(mode)
            bpr = 24.5 if info[name]["nibble"] else 26.0
            rec = dict(march_info=info[name], bytes_per_row=bpr)
            for w, k in ((1, "P"), (2, "B"), (5, "iteration")):
                ms = best[(name, w)]
                by = bpr * N * (2 if w == 5 else 1)
                rec[k] = dict(ms=round(ms, 5), gbs=round(by / (ms * 1e-3) / 1e9, 1),
                              frac=round(by / (ms * 1e-3) / 8e12, 4))
            t = {}
            for n in (args.iters // 2, args.iters):
                t0 = time.perf_counter()
                it = ctx.conductance(*rule, tol=0.0, itmax=n - 1)["iter"]
                t[n] = (time.perf_counter() - t0, it)
            (t1, i1), (t2, i2) = t[args.iters // 2], t[args.iters]
            rec["solve_ms_per_it"] = round((t2 - t1) * 1e3 / (i2 - i1), 5)
            out[name] = rec
    out.update(N=N, kind=args.kind, p=args.p, ps=args.ps if args.kind != "bond" else None)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
