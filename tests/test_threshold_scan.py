"""Threshold scans (Fortran/Square/bond_perc.f, site_perc.f and their
Triangular twins): per trial, the first occupation count with a spanning
cluster and the cluster sizes at that step, against the reference's
bond_perc.txt / site_perc.txt (tests/golden, made by the compiled reference).

* CPU: the algorithm -- tseed scale 1e6, the reference shuffle, bisection
  over counts (spanning is monotone), label replay at the first spanning
  count -- with the host replay as the spanning test.
* GPU: perc_first_spanning (GPU labeling inside the bisection) through
  api.threshold_scan, byte-identical text.
"""
import numpy as np
import pytest

import golden_io as G
from percolation_amd import _lib as PL
from percolation_amd import api

VARIANTS = [v for v in G.variants() if G.meta(v)["kind"] in ("bond_perc", "site_perc")]


def kind_of(v):
    return PL.BOND if G.meta(v)["kind"] == "bond_perc" else PL.SITE


def fname(v):
    return G.meta(v)["kind"] + ".txt"


def replay(p, kind, order, c):
    if kind == PL.BOND:
        return api.replay_labels(p["lattice"], p["m"], p["n"], p["pbc"], kind, bond_order=order,
                                 nbond=c)
    return api.replay_labels(p["lattice"], p["m"], p["n"], p["pbc"], kind, site_order=order,
                             nsites=c)


@pytest.mark.parametrize("v", VARIANTS)
def test_threshold_scan_host_replay(v):
    p = G.meta(v)["params"]
    kind = kind_of(v)
    N = api.nbonds(p["lattice"], p["m"], p["n"], p["pbc"]) if kind == PL.BOND else p["m"] * p["n"]
    seeds = api.trial_seeds(p["seed"], p["numtrials"], scale=1000000)
    rows = []
    for ii in range(p["numtrials"]):
        order = api.shuffled_ids(N, int(seeds[ii]))
        lo, hi = 0, N
        if replay(p, kind, order, N)["perccln"] == 0:
            hi = 0
        while hi and hi - lo > 1:
            mid = (lo + hi) // 2
            if replay(p, kind, order, mid)["perccln"]:
                hi = mid
            else:
                lo = mid
        c = hi or N
        r = replay(p, kind, order, c)
        rows.append(dict(tseed=int(seeds[ii]), f=float(np.float32(np.float32(c) / np.float32(N))),
                         maxcs=r["maxcs"], perccls=int(r["csize"][r["perccln"]]) if hi else 0))
    assert api.fmt_perc_rows(rows).encode() == G.text(v, fname(v))


@pytest.mark.gpu
@pytest.mark.parametrize("v", VARIANTS)
def test_threshold_scan_gpu(v):
    p = G.meta(v)["params"]
    rows = api.threshold_scan(p["lattice"], p["m"], p["n"], p["pbc"], kind_of(v), p["seed"],
                              p["numtrials"])
    assert api.fmt_perc_rows(rows).encode() == G.text(v, fname(v))
