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


# ---------------------------------------------------------------- mixed scans
MIXED = [v for v in G.variants() if G.meta(v)["kind"] in ("sb_perc", "bs_perc")]


def mixed_rows(v, first_of):
    """sb_perc / bs_perc records with the first spanning count from first_of(
    scan, so, fixed-count, bo, N)."""
    md = G.meta(v)
    p = md["params"]
    lat, m, n, pbc = p["lattice"], p["m"], p["n"], p["pbc"]
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    scan_b = md["kind"] == "sb_perc"
    pseed = api.trial_seeds(p["seed"], 100)
    rows = []
    for ii, pt in enumerate(p["points"]):
        ss, bs = api.paired_seeds(pseed[ii])
        for jj in range(p["iters"]):
            so, bo = api.shuffled_ids(t, int(ss[jj])), api.shuffled_ids(nb, int(bs[jj]))
            fixed = int(pt * (t if scan_b else nb))
            first = first_of(scan_b, so, fixed, bo)
            N, F = (nb, t) if scan_b else (t, nb)
            f = float(np.float32(first) / np.float32(N)) if first else 0.0
            fx = float(np.float32(fixed) / np.float32(F))
            rows.append(dict(sseed=int(ss[jj]), bseed=int(bs[jj]), ps=fx if scan_b else f,
                             pb=f if scan_b else fx))
    return rows


@pytest.mark.parametrize("v", MIXED)
def test_mixed_scan_host(v):
    """sb_perc: bisection with the host sitebond replay as the spanning test;
    bs_perc: the as-built replay (hazard H11)."""
    p = G.meta(v)["params"]
    lat, m, n, pbc = p["lattice"], p["m"], p["n"], p["pbc"]
    t, nb = m * n, api.nbonds(lat, m, n, pbc)

    def first_of(scan_b, so, fixed, bo):
        if not scan_b:
            return api.bs_perc_replay(lat, m, n, pbc, so, t, bo, fixed, True)

        def spans(c):
            return api.replay_labels(lat, m, n, pbc, PL.SITEBOND, site_order=so, nsites=fixed,
                                     bond_order=bo, nbond=c)["perccln"] > 0
        lo, hi = 0, nb
        if not spans(nb):
            return 0
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if spans(mid):
                hi = mid
            else:
                lo = mid
        return hi
    assert api.fmt_mixed_rows(mixed_rows(v, first_of)).encode() == \
        G.text(v, G.meta(v)["kind"] + ".txt")


def test_bs_perc_intended_rule_is_connectivity():
    """Without the c(0) overflow the bs_perc replay is plain site+bond
    connectivity: its first spanning count equals the sitebond replay's."""
    lat, m, n, pbc = 0, 12, 12, 0
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    for seed in range(1, 25):
        so, bo = api.shuffled_ids(t, seed), api.shuffled_ids(nb, seed + 1000)
        tb = int(0.7 * nb)
        first = api.bs_perc_replay(lat, m, n, pbc, so, t, bo, tb, False)
        c = next((c for c in range(1, t + 1)
                  if api.replay_labels(lat, m, n, pbc, PL.SITEBOND, site_order=so, nsites=c,
                                       bond_order=bo, nbond=tb)["perccln"] > 0), 0)
        assert first == c, seed


@pytest.mark.gpu
@pytest.mark.parametrize("v", MIXED)
def test_mixed_scan_gpu(v):
    md = G.meta(v)
    p = md["params"]
    rows = api.mixed_scan(p["lattice"], p["m"], p["n"], p["pbc"],
                          PL.BOND if md["kind"] == "sb_perc" else PL.SITE, p["seed"],
                          p["points"], p["iters"])
    assert api.fmt_mixed_rows(rows).encode() == G.text(v, md["kind"] + ".txt")


@pytest.mark.gpu
def test_bs_scan_gpu_intended_equals_replay():
    lat, m, n, pbc = 1, 20, 16, 1
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    with api.Context(lat, m, n, pbc) as ctx:
        for seed in range(1, 12):
            so, bo = api.shuffled_ids(t, seed), api.shuffled_ids(nb, seed + 77)
            tb = int(0.6 * nb)
            assert api.first_spanning_mixed(ctx, PL.SITE, so, t, bo, tb) == \
                api.bs_perc_replay(lat, m, n, pbc, so, t, bo, tb, False)


# ---------------------------------------------------------------- GPU cluster sizes
@pytest.mark.gpu
@pytest.mark.parametrize("lat,m,n,pbc", [(0, 64, 64, 0), (0, 100, 70, 1), (1, 64, 80, 0),
                                         (1, 90, 64, 1), (0, 512, 512, 0)])
@pytest.mark.parametrize("kind", [PL.BOND, PL.SITE])
def test_cluster_sizes_equal_replay(lat, m, n, pbc, kind):
    """perc_cluster_sizes (GPU) = the reference's maxcs (running maximum of
    c(label), bond_perc.f:313-322) and c(perccln) of the lowest-label
    spanning cluster, by the host replay, at counts below, at and above the
    threshold."""
    N = api.nbonds(lat, m, n, pbc) if kind == PL.BOND else m * n
    order = api.shuffled_ids(N, 4242 + m + n)
    pcs = (0.3, 0.45, 0.5, 0.55, 0.7, 1.0) if kind == PL.BOND else (0.4, 0.55, 0.6, 0.65, 0.8)
    if lat == 1:
        pcs = tuple(p - 0.15 if kind == PL.BOND else p - 0.1 for p in pcs)
    with api.Context(lat, m, n, pbc) as ctx:
        for p in pcs:
            c = int(p * N)
            if kind == PL.BOND:
                ctx.occupy(kind, bond_order=order, nbonds_=c)
            else:
                ctx.occupy(kind, site_order=order, nsites=c)
            li = ctx.label()
            mx, sp = ctx.cluster_sizes()
            r = replay({"lattice": lat, "m": m, "n": n, "pbc": pbc}, kind, order, c)
            assert mx == r["maxcs"], (p, mx, r["maxcs"])
            want = int(r["csize"][r["perccln"]]) if r["perccln"] > 0 else 0
            assert (li["nspan"] > 0) == (r["perccln"] > 0)
            assert sp == want, (p, sp, want)
