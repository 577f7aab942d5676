#!/usr/bin/env python3
"""Slot-weighted band weights of the strip-major march (perc_set_band_weights)
on the metric realisation: per-kernel launch times inside fixed-iteration
solves (perc_set_kernel_timing: dispatch timestamps of every 8th launch -- PERC_TIME_EVERY=8, P
and B alternating as in the bench) and the solve's ms per iteration, for
each pair of candidate weight sets (P set i with B set i), the pairs
interleaved round after round so box drift hits them alike; median and best
per pair.  The march trace of round 5 (profiles/r5_4_mtrace_summary_L4096.txt)
put P's third CU slot and B's first ~2-3 us above the others' mean walk: the
weights decide how many rows each slot's bands get.

  python tools/weights_probe.py --rounds 7 --iters 2000
  python tools/weights_probe.py --p-sets 100,75,50:100,77,47 --b-sets 100,80,60:100,84,63
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def parse_sets(s):
    return [tuple(int(x) for x in part.split(",")) for part in s.split(":") if part]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--tseed", type=int, default=9161242)  # the bench's first realisation
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--p-sets", default="100,75,50:100,76,48:100,77,46:100,78,48:100,74,46:100,76,50")
    ap.add_argument("--b-sets", default="100,80,60:100,84,63:100,82,62:100,86,65:100,83,60:100,85,67")
    args = ap.parse_args()
    os.environ.setdefault("PERC_TIME_EVERY", "8")  # (more samples per short solve than the bench's 64)
    from percolation_amd import _lib as PL
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    psets, bsets = parse_sets(args.p_sets), parse_sets(args.b_sets)
    assert len(psets) == len(bsets), "P and B sets are run in pairs"
    pairs = list(zip(psets, bsets))
    res = {pr: dict(P=[], B=[], it=[]) for pr in pairs}
    import time
    with api.Context(0, L_, L_, 0) as ctx:
        ctx.occupy_random(PL.BOND, 0, int(args.p * nb), args.tseed)
        assert ctx.label()["nspan"] > 0
        ctx.conductance(tol=1e-8, itmax=50)  # assembled, solver state warm
        info = ctx.march_info()
        for rnd in range(args.rounds):
            for pw, bw in pairs:
                ctx.set_band_weights(0, list(pw))
                ctx.set_band_weights(1, list(bw))
                ctx.set_kernel_timing(True)
                ctx.kernel_stats(reset=True)
                t0 = time.perf_counter()
                c = ctx.conductance(tol=0.0, itmax=args.iters - 1)
                dt = time.perf_counter() - t0
                ks = ctx.kernel_stats(reset=True)
                ctx.set_kernel_timing(False)
                r = res[(pw, bw)]
                r["P"].append(ks["spmv_ms"] / max(ks["spmv_n"], 1))
                r["B"].append(ks["resid_ms"] / max(ks["resid_n"], 1))
                r["it"].append(dt * 1e3 / max(c["iter"], 1))
            ctx.set_band_weights()
            print("round %d done" % rnd, file=sys.stderr, flush=True)
    out = dict(L=L_, p=args.p, tseed=args.tseed, rounds=args.rounds, iters=args.iters, march_info=info,
               pairs=[])
    for (pw, bw), r in res.items():
        out["pairs"].append(dict(p_weights=list(pw), b_weights=list(bw),
                                 **{k + "_median_ms": round(statistics.median(v), 5) for k, v in r.items()},
                                 **{k + "_best_ms": round(min(v), 5) for k, v in r.items()}))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
