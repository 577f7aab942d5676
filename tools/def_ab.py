#!/usr/bin/env python3
"""Deferred march reductions (k_cg_march DEF, the default) against the
end-of-launch collectors (PERC_MARCH_NODEF=1) on the metric realisation:

  * the full solve at the reference tolerance in both forms -- the same
    association, so iter, err, Gtop and Gbot must be identical;
  * interleaved rounds of fixed-iteration solves with live kernel timing
    (perc_set_kernel_timing): P and B average launch times and ms per
    iteration, median and best per form.

  python tools/def_ab.py --rounds 7 --iters 3000
  python tools/def_ab.py --forms "def3=PERC_MARCH_DEF:3;def1=PERC_MARCH_DEF:1;coll=PERC_MARCH_NODEF:1" \
      --p-weights 100,76,48
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--tseed", type=int, default=9161242)  # the bench's first realisation
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--full", type=int, default=1, help="also the full solve at tol 1e-8 in every form")
    ap.add_argument("--forms", default="deferred=PERC_MARCH_NODEF:0;collectors=PERC_MARCH_NODEF:1",
                    help="name=VAR:value,VAR:value;... (environment of each form)")
    ap.add_argument("--p-weights", default="", help="band weights of P (perc_set_band_weights 0)")
    ap.add_argument("--b-weights", default="", help="band weights of B (perc_set_band_weights 1)")
    args = ap.parse_args()
    from percolation_amd import _lib as PL
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    forms = {}
    for part in args.forms.split(";"):
        name, _, envs = part.partition("=")
        forms[name] = dict(e.split(":") for e in envs.split(",") if e)
    knobs = sorted({k for env in forms.values() for k in env})

    def use(f):
        for k in knobs:
            os.environ.pop(k, None)
        os.environ.update(forms[f])
    res = {f: dict(P=[], B=[], it=[]) for f in forms}
    out = dict(L=L_, p=args.p, tseed=args.tseed, rounds=args.rounds, iters=args.iters)
    with api.Context(0, L_, L_, 0) as ctx:
        ctx.occupy_random(PL.BOND, 0, int(args.p * nb), args.tseed)
        assert ctx.label()["nspan"] > 0
        if args.p_weights:
            ctx.set_band_weights(0, [int(x) for x in args.p_weights.split(",")])
        if args.b_weights:
            ctx.set_band_weights(1, [int(x) for x in args.b_weights.split(",")])
        out.update(p_weights=args.p_weights, b_weights=args.b_weights, forms_env=forms)
        if args.full:
            full = {}
            for f in forms:
                use(f)
                t0 = time.perf_counter()
                c = ctx.conductance(tol=1e-8, itmax=10 ** 6)
                full[f] = dict(iter=c["iter"], err=repr(c["err"]), gtop=repr(c["gtop"]), gbot=repr(c["gbot"]),
                               ran=ctx.last_solve(), seconds=round(time.perf_counter() - t0, 3))
                print(f, json.dumps(full[f]), file=sys.stderr, flush=True)
            first = full[next(iter(forms))]
            full["identical"] = all(all(v[k] == first[k] for k in ("iter", "err", "gtop", "gbot"))
                                    for v in full.values())
            out["full_solve"] = full
        for rnd in range(args.rounds):
            for f in forms:
                use(f)
                ctx.set_kernel_timing(True)
                ctx.kernel_stats(reset=True)
                t0 = time.perf_counter()
                c = ctx.conductance(tol=0.0, itmax=args.iters - 1)
                dt = time.perf_counter() - t0
                ks = ctx.kernel_stats(reset=True)
                ctx.set_kernel_timing(False)
                r = res[f]
                r["P"].append(ks["spmv_ms"] / max(ks["spmv_n"], 1))
                r["B"].append(ks["resid_ms"] / max(ks["resid_n"], 1))
                r["it"].append(dt * 1e3 / max(c["iter"], 1))
            print("round %d: %s" % (rnd, {f: round(res[f]["it"][-1], 5) for f in forms}), file=sys.stderr,
                  flush=True)
    for k in knobs:
        os.environ.pop(k, None)
    out["forms"] = {f: {k + "_median_ms": round(statistics.median(v), 5) for k, v in r.items()} |
                    {k + "_best_ms": round(min(v), 5) for k, v in r.items()} for f, r in res.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
