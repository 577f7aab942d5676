#!/usr/bin/env python3
"""The literal dot order at a BASELINE config size against the committed
oracle fixture (tests/golden/configs/<case>.json, the oracle's literal
linbcg -- bitwise the reference solver at <= 64^2).

With perc_set_dot_order(PERC_DOT_LITERAL) the GPU folds linbcg's three dot
products in ascending j (Square/bondc.f:785-787, 803-805, 872-875); every
other operation is already the reference's, so Gtop, Gbot, iter, err and the
fixture's decimated err history must match bitwise.  The solve runs the
production kernels, which store their rows' dot terms for the folds:
--solver resident (k_cg_res, the default solver of configs 2-4) or march (the
q-free strip-major march P / B of the metric; PERC_SOLVE_RESIDENT off), or
march_host (the same march, PERC_DOT_LITERAL_HOST: the serial sums formed by
the host CPU from the kernels' terms -- bitwise the GPU fold, ~4x faster);
perc_last_solve's record is printed with each result.  Prints one JSON line
per tolerance; exit status 1 on any difference.

  python tools/literal_config.py c2_sq1024_bond_p50 --tol 1e-08 [--solver march]
  python tools/literal_config.py c4_sq2048_bond_p50 --probe 300   # ms per iteration,
      # and the fixture's err-history points within the first 300 iterations
"""
import argparse
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from percolation_amd import _lib as PL  # noqa: E402
from percolation_amd import api  # noqa: E402
from test_config_goldens import occupation  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--tol", action="append", default=None)
    ap.add_argument("--solver", default="resident", choices=("resident", "march", "march_host"),
                    help="march_host: the march with PERC_DOT_LITERAL_HOST (sums folded by the host CPU)")
    ap.add_argument("--probe", type=int, default=0,
                    help="run this many iterations (tol 1e-300) and compare the history prefix")
    args = ap.parse_args()
    tols = args.tol or ["1e-08"]
    # a heartbeat on stderr while a solve runs (minutes in the literal order)
    t_start = time.time()
    stop = threading.Event()

    def beat():
        while not stop.wait(30.0):
            print("... %.0f s" % (time.time() - t_start), file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    doc = json.load(open(os.path.join(REPO, "tests", "golden", "configs", args.case + ".json")))
    rc = doc["recipe"]
    occ, rule, cur = occupation(rc)
    ok = True
    with api.Context(rc["lattice"], rc["L"], rc["L"], 0) as ctx:
        if args.solver != "resident":
            ctx.set_march_mode(PL.MARCH_DEFAULT & ~PL.SOLVE_RESIDENT)
        if "device" in occ:  # drawn on the GPU (the bench realisation's fixture)
            ctx.occupy_random(*occ["device"])
        else:
            ctx.occupy(**occ)
        li = ctx.label()
        assert li["nspan"] > 0
        ctx.set_dot_order(PL.DOT_LITERAL_HOST if args.solver == "march_host" else PL.DOT_LITERAL)
        if args.probe:
            ref = doc["solves"][tols[0]]
            t0 = time.time()
            c = ctx.conductance(rule, cur, tol=1e-300, itmax=args.probe - 1)
            secs = time.time() - t0
            hist = ctx.err_history()
            want = [(k, e) for k, e in ref["err_history"] if k <= c["iter"]]
            same = all(hist[k - 1] == e for k, e in want)
            ok = same
            print(json.dumps(dict(case=args.case, probe_iterations=c["iter"], solver=args.solver,
                                  ran=ctx.last_solve(), err_history_points=len(want),
                                  err_history_bitwise=same, seconds=round(secs, 2),
                                  ms_per_iteration=round(secs * 1e3 / max(c["iter"], 1), 3))), flush=True)
        for tkey in ([] if args.probe else tols):
            ref = doc["solves"][tkey]
            t0 = time.time()
            c = ctx.conductance(rule, cur, tol=float(tkey), itmax=10 ** 6)
            secs = time.time() - t0
            hist = ctx.err_history()
            want = ref["err_history"]
            hist_ok = all(hist[k - 1] == e for k, e in want)
            same = (c["iter"] == ref["iter"] and c["err"] == ref["err"] and c["gtop"] == ref["gtop"]
                    and c["gbot"] == ref["gbot"] and hist_ok)
            ok = ok and same
            print(json.dumps(dict(case=args.case, tol=tkey, solver=args.solver, ran=ctx.last_solve(),
                                  bitwise=same, iter=c["iter"], iter_ref=ref["iter"],
                                  gtop=repr(c["gtop"]), gtop_ref=repr(ref["gtop"]), gbot=repr(c["gbot"]),
                                  gbot_ref=repr(ref["gbot"]), err=repr(c["err"]), err_ref=repr(ref["err"]),
                                  err_history_points=len(want), err_history_bitwise=hist_ok,
                                  seconds=round(secs, 1),
                                  ms_per_iteration=round(secs * 1e3 / max(c["iter"], 1), 3))),
                  flush=True)
    stop.set()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
