"""GPU parity: libperc's HIP path against the oracle and the reference goldens.

Bars: partitions bit-exact (canonical ids), assembled
system and SpMV bitwise, CG iteration count within +-1 of the reference's,
Gtop within 1e-10 relative at the reference settings (tol 1e-8), Gtop and
Gbot within 1e-10 relative when both sides solve to tol 1e-14.
"""
import ctypes as C

import numpy as np
import pytest

import golden_io as G
import oracle_lib as O
import percolation_amd as P
from percolation_amd import _lib as PL
from percolation_amd import api

pytestmark = pytest.mark.gpu
REL = 1e-10


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


# ------------------------------------------------------------ helpers
def oracle_canon_bonds(b1, b2, label, t):
    """per-site canonical id (min site of the component) from bond labels"""
    canon = np.zeros(t, np.int64)
    lab = label.astype(np.int64)
    occ = lab > 0
    if not occ.any():
        return canon
    big = np.iinfo(np.int64).max
    mins = np.full(lab.max() + 1, big)
    np.minimum.at(mins, lab[occ], b1[occ])
    for arr in (b1, b2):
        np.maximum.at(canon, arr[occ] - 1, mins[lab[occ]])
    return canon


def oracle_canon_sites(s):
    t = len(s)
    canon = np.zeros(t, np.int64)
    occ = s > 0
    big = np.iinfo(np.int64).max
    mins = np.full(s.max() + 1 if occ.any() else 1, big)
    sites = np.arange(1, t + 1)
    np.minimum.at(mins, s[occ], sites[occ])
    canon[occ] = mins[s[occ]]
    return canon


# ------------------------------------------------------------ labeling
BOND_CASES = [(0, 64, 64, 0, 0.5, 1), (0, 128, 96, 1, 0.52, 2), (1, 64, 64, 0, 0.35, 3),
              (1, 100, 80, 1, 0.33, 4), (0, 256, 256, 0, 0.5, 5), (0, 256, 256, 0, 0.7, 6)]


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", BOND_CASES)
def test_bond_partition_bitexact(lat, m, n, pbc, p, seed):
    b1, b2 = api.bond_list(lat, m, n, pbc)
    nb = len(b1)
    order = api.shuffled_ids(nb, seed)
    tb = int(p * nb)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        li = ctx.label(canon=True)
        ref = api.replay_labels(lat, m, n, pbc, PL.BOND, bond_order=order, nbond=tb)
        want = oracle_canon_bonds(b1, b2, ref["bond_label"], m * n)
        assert np.array_equal(li["canon"].astype(np.int64), want)
        # spanning agrees with the reference rule
        assert (li["nspan"] > 0) == (ref["perccln"] > 0)
        if li["nspan"] == 1:
            k = np.nonzero(ref["bond_label"] == ref["perccln"])[0][0]
            assert li["span_root"] == want[b1[k] - 1]


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", [(0, 64, 64, 0, 0.6, 7), (1, 64, 64, 0, 0.5, 8),
                                                 (0, 200, 150, 1, 0.59, 9),
                                                 (1, 128, 128, 1, 0.5, 10)])
def test_site_partition_bitexact(lat, m, n, pbc, p, seed):
    t = m * n
    order = api.shuffled_ids(t, seed)
    ts = int(p * t)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.SITE, site_order=order, nsites=ts)
        li = ctx.label(canon=True)
    ref = api.replay_labels(lat, m, n, pbc, PL.SITE, site_order=order, nsites=ts)
    assert np.array_equal(li["canon"].astype(np.int64), oracle_canon_sites(ref["site_label"]))
    assert (li["nspan"] > 0) == (ref["perccln"] > 0)


@pytest.mark.parametrize("lat,m,n,pbc,ps,pb,seed", [(0, 64, 64, 0, 0.9, 0.6, 11),
                                                     (1, 64, 64, 0, 0.8, 0.5, 12),
                                                     (0, 128, 128, 0, 0.593, 1.0, 13)])
def test_sitebond_partition_bitexact(lat, m, n, pbc, ps, pb, seed):
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    so, bo = api.shuffled_ids(t, seed), api.shuffled_ids(nb, seed + 1)
    ts, tb = int(ps * t), int(pb * nb)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.SITEBOND, site_order=so, nsites=ts, bond_order=bo, nbonds_=tb)
        li = ctx.label(canon=True)
    ref = api.replay_labels(lat, m, n, pbc, PL.SITEBOND, site_order=so, nsites=ts, bond_order=bo,
                            nbond=tb)
    assert np.array_equal(li["canon"].astype(np.int64), oracle_canon_sites(ref["site_label"]))
    assert (li["nspan"] > 0) == (ref["perccln"] > 0)


@pytest.mark.parametrize("lat,m,n,pbc,ps,pb,seed", [(0, 30, 30, 1, 0.8, 0.7, 21),
                                                     (1, 64, 48, 0, 0.7, 0.6, 22),
                                                     (0, 128, 96, 0, 0.85, 0.75, 23)])
def test_bondsite_site_partition_matches_gpu(lat, m, n, pbc, ps, pb, seed):
    """bondsite (bonds first, then sites) connects two sites exactly when an
    occupied bond joins them, as the GPU mixed labeling does: the site
    partition of the PERC_BONDSITE replay equals the GPU's (canonical
    min-site ids), whatever the history-dependent numbering."""
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    so, bo = api.shuffled_ids(t, seed), api.shuffled_ids(nb, seed + 1)
    ts, tb = int(ps * t), int(pb * nb)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.SITEBOND, site_order=so, nsites=ts, bond_order=bo, nbonds_=tb)
        li = ctx.label(canon=True)
    ref = api.replay_labels(lat, m, n, pbc, PL.BONDSITE, site_order=so, nsites=ts,
                            bond_order=bo, nbond=tb)
    assert np.array_equal(li["canon"].astype(np.int64), oracle_canon_sites(ref["site_label"]))


# ------------------------------------------------------------ assembly + SpMV
def oracle_system(lat, m, n, pbc, b1, b2, gval):
    t, N = m * n, m * n - 2 * m
    nmax = N + 1 + 2 * len(b1) + 8
    sa, ija = O.f64(nmax), O.i32(nmax)
    itemp, diag = O.f64(N), O.f64(t)
    k = O.lib().or_assemble(lat, m, n, pbc, len(b1), b1, b2, gval, 1.0, 1e-16, 0, nmax, sa, ija,
                            itemp, diag)
    return sa, ija, itemp, diag, k


FORMATS = [PL.FMT_STENCIL, PL.FMT_STENCIL_TILED, PL.FMT_STENCIL_SPLIT, PL.FMT_CSR]


def used_fmt(fmt, m):
    """The format perc_matrix_format reports for a request: PERC_FMT_STENCIL
    runs the register-march kernel when m is a multiple of 128, else the
    LDS-tiled one."""
    return PL.FMT_STENCIL_TILED if fmt == PL.FMT_STENCIL and m % 128 else fmt


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("lat,m,n,pbc,p,seed", BOND_CASES[:4])
def test_assembly_and_spmv_bitwise(lat, m, n, pbc, p, seed, fmt):
    b1, b2 = api.bond_list(lat, m, n, pbc)
    nb = len(b1)
    order = api.shuffled_ids(nb, seed)
    tb = int(max(p, 0.6 if lat == 0 else 0.4) * nb)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        li = ctx.label()
        assert li["nspan"] >= 1
        ctx.set_matrix_format(fmt)
        ctx.conductance(itmax=3)
        assert ctx.matrix_format() == used_fmt(fmt, m)
        sysm = ctx.system()
        ref = api.replay_labels(lat, m, n, pbc, PL.BOND, bond_order=order, nbond=tb)
        gval = O.f64(nb)
        O.lib().or_bond_values(0, nb, b1, b2, ref["bond_label"], O.i32(1), ref["perccln"], 1.0,
                               1e-12, gval)
        sa, ija, itemp, diag, k = oracle_system(lat, m, n, pbc, b1, b2, gval)
        N = m * n - 2 * m
        # NR layout -> CSR
        rp = ija[:N + 1] - (N + 2)
        assert np.array_equal(sysm["rowptr"], rp)
        assert np.array_equal(sysm["col"], ija[N + 1:k] - 1)
        assert np.array_equal(sysm["val"].view(np.uint64), sa[N + 1:k].view(np.uint64))
        assert np.array_equal(sysm["diag"].view(np.uint64), sa[:N].view(np.uint64))
        assert np.array_equal(sysm["rhs"].view(np.uint64), itemp.view(np.uint64))
        x = np.random.default_rng(seed).standard_normal(N)
        y = ctx.spmv(x)
        yo = O.f64(N)
        O.lib().or_dsprsax(sa, ija, x, yo, N)
        assert np.array_equal(y.view(np.uint64), yo.view(np.uint64))


# ------------------------------------------------------------ conductance
BONDC = [v for v in G.variants() if G.meta(v)["kind"] == "bondc" and G.meta(v)["perccln"]]


@pytest.mark.parametrize("v", BONDC)
def test_bondc_against_reference(v):
    md = G.meta(v)
    p = md["params"]
    tol, itmax = p.get("tol", 1e-8), p.get("itmax", 2500)
    r = api.bondc(p["lattice"], p["m"], p["n"], p["pbc"], p["pb"], p["seed"], tol=tol,
                  itmax=itmax)
    assert r["perccln"] == md["perccln"] and r["perccls"] == md["perccls"]
    assert abs(r["iter"] - md["iter"]) <= 1, (r["iter"], md["iter"])
    assert rel(r["gtop"], md["gtop"]) < REL, (r["gtop"], md["gtop"])
    if tol <= 1e-13:
        assert rel(r["gbot"], md["gbot"]) < REL, (r["gbot"], md["gbot"])
    else:
        # the reference's own Gbot at tol 1e-8 is off the converged value by
        # up to ~3e-7 (SURVEY.md §7 hard part 2): compare at that scale
        assert rel(r["gbot"], md["gbot"]) < 1e-6


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("lat,m,n,p,seed", [(0, 128, 128, 0.6, 21), (1, 96, 96, 0.4, 22),
                                            (0, 200, 160, 0.55, 23)])
def test_conductance_vs_oracle_linbcg(lat, m, n, p, seed, fmt):
    """Larger lattices: oracle literal linbcg (CPU) vs fused GPU PCG."""
    b1, b2 = api.bond_list(lat, m, n, 0)
    nb = len(b1)
    order = api.shuffled_ids(nb, seed)
    tb = int(p * nb)
    ref = api.replay_labels(lat, m, n, 0, PL.BOND, bond_order=order, nbond=tb)
    assert ref["perccln"] > 0
    gval = O.f64(nb)
    O.lib().or_bond_values(0, nb, b1, b2, ref["bond_label"], O.i32(1), ref["perccln"], 1.0, 1e-12,
                           gval)
    oc = O.conductance(lat, m, n, 0, b1, b2, gval, itmax=100000)
    ot = O.conductance(lat, m, n, 0, b1, b2, gval, tol=1e-13, itmax=100000)
    with api.Context(lat, m, n, 0) as ctx:
        ctx.set_matrix_format(fmt)
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        c = ctx.conductance(itmax=100000, vint=True)
        assert ctx.matrix_format() == used_fmt(fmt, m)
        ct = ctx.conductance(tol=1e-13, itmax=100000)
    # reference settings: same iteration count, answers agree to the solver
    # tolerance (the two differ only in the association of the dot products)
    assert abs(c["iter"] - oc["iter"]) <= 1
    assert rel(c["gtop"], oc["gtop"]) < 1e-8
    # voltages: tight on the spanning cluster's sites; nodes coupled only by
    # the 1e-12 leak are barely constrained by the residual norm at tol 1e-8
    # and agree to that scale only (their drift depends on the dot-product
    # association)
    t = m * n
    on = np.zeros(t + 1, bool)
    sel = ref["bond_label"] == ref["perccln"]
    on[b1[sel]] = True
    on[b2[sel]] = True
    span = on[m + 1:t - m + 1]
    dv = np.abs(c["vint"] - oc["vint"])
    assert np.max(dv[span]) < 1e-6, np.max(dv[span])
    assert np.max(dv) < 1e-3
    # converged: Gtop and Gbot to 1e-10
    assert rel(ct["gtop"], ot["gtop"]) < REL and rel(ct["gbot"], ot["gbot"]) < REL


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 300, 200, 0, 0.6), (0, 128, 96, 1, 0.55),
                                           (1, 160, 120, 0, 0.4), (1, 128, 100, 1, 0.42),
                                           # tile edges: m past one 256-column tile, rows
                                           # not a multiple of 16, tiny pbc widths
                                           (0, 520, 37, 1, 0.55), (1, 514, 30, 1, 0.42),
                                           (0, 24, 50, 1, 0.55), (1, 20, 18, 0, 0.45),
                                           # register-march kernel: several strips,
                                           # pbc wrap columns, triangular forms
                                           (0, 256, 77, 0, 0.6), (1, 384, 50, 1, 0.42),
                                           (0, 128, 300, 1, 0.55)])
def test_stencil_matches_csr_solver(lat, m, n, pbc, p):
    """The stencil operator (fused LDS-tiled and split kernels) rebuilds the
    CSR numbers bitwise, so all formats give the same iterates up to the
    association of the q.p dot (its per-thread row order differs): same
    iteration count within 1, Gtop and the voltages to the solver's
    precision, and bitwise-equal SpMVs."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 777)
    out = {}
    x = np.random.default_rng(5).standard_normal(m * n - 2 * m)
    for fmt in FORMATS:
        with api.Context(lat, m, n, pbc) as ctx:
            ctx.set_matrix_format(fmt)
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
            if ctx.label()["nspan"] == 0:
                pytest.skip("no spanning cluster")
            c = ctx.conductance(tol=1e-12, itmax=100000, vint=True)
            assert ctx.matrix_format() == used_fmt(fmt, m)
            out[fmt] = (c, ctx.spmv(x))
    cc, yc = out[PL.FMT_CSR]
    for fmt in (PL.FMT_STENCIL, PL.FMT_STENCIL_TILED, PL.FMT_STENCIL_SPLIT):
        cs, ys = out[fmt]
        assert np.array_equal(ys.view(np.uint64), yc.view(np.uint64))
        assert abs(cs["iter"] - cc["iter"]) <= 1
        assert rel(cs["gtop"], cc["gtop"]) < REL and rel(cs["gbot"], cc["gbot"]) < REL
        assert np.max(np.abs(cs["vint"] - cc["vint"])) < 1e-6


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 260, 140, 0, 0.6), (1, 130, 90, 1, 0.42),
                                           (0, 256, 140, 0, 0.6), (1, 128, 90, 1, 0.42)])
def test_boundary_row_voltages_bitwise(lat, m, n, pbc, p, fmt):
    """Without vint_out the solver keeps x on the two interior rows next to
    the electrodes only; Gtop/Gbot/iter/err are bitwise those of the
    full-voltage solve, and those rows' voltages too."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 4242)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.set_matrix_format(fmt)
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        part = ctx.conductance(tol=1e-10, itmax=100000)
        ctx.set_full_voltages(True)
        full = ctx.conductance(tol=1e-10, itmax=100000)
        vfull = ctx.conductance(tol=1e-10, itmax=100000, vint=True)["vint"]
        ctx.set_full_voltages(False)
        vpart = ctx.conductance(tol=1e-10, itmax=100000, vint=True)["vint"]
    for k in ("gtop", "gbot", "err", "iter"):
        assert part[k] == full[k], k
    assert np.array_equal(vfull.view(np.uint64), vpart.view(np.uint64))  # vint forces all rows


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 2048, 2048, 0, 0.6), (1, 1024, 2050, 1, 0.42)])
def test_tall_tiles_match_split_kernels(lat, m, n, pbc, p):
    """Lattices large enough for the 32-row (2048^2) and 16-row (1024 x 2050)
    tiles of the fused kernel: same solve as the split stencil kernels."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 99)
    out = {}
    for fmt in (PL.FMT_STENCIL, PL.FMT_STENCIL_SPLIT):
        with api.Context(lat, m, n, pbc) as ctx:
            ctx.set_matrix_format(fmt)
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
            if ctx.label()["nspan"] == 0:
                pytest.skip("no spanning cluster")
            out[fmt] = ctx.conductance(tol=1e-10, itmax=10 ** 6)
            assert ctx.matrix_format() == used_fmt(fmt, m)
    a, b = out[PL.FMT_STENCIL], out[PL.FMT_STENCIL_SPLIT]
    assert abs(a["iter"] - b["iter"]) <= 2
    assert rel(a["gtop"], b["gtop"]) < REL and rel(a["gbot"], b["gbot"]) < REL


def test_site_and_mixed_rules_vs_direct_solve():
    """ConductCalc.m site / mixed rules (parity unpinned vs MATLAB: checked
    against an independent direct sparse solve of the oracle's system)."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    for kind, rule, lat, m, n in [(PL.SITE, PL.RULE_SITE, 0, 64, 64),
                                  (PL.SITE, PL.RULE_SITE, 1, 64, 64),
                                  (PL.SITEBOND, PL.RULE_MIXED, 0, 64, 64)]:
        t = m * n
        b1, b2 = api.bond_list(lat, m, n, 0)
        nb = len(b1)
        if kind == PL.SITE:
            r = api.site(lat, m, n, 0, ps=0.66 if lat == 0 else 0.60, seed=1080115,
                         conductance=True, tol=1e-14, itmax=200000)
            s, bl = r["site_label"], O.i32(nb)
        else:
            r = api.sitebond(lat, m, n, 0, ps=0.95, pb=0.75, conductance=True, tol=1e-14,
                             itmax=200000)
            s, bl = r["site_label"], r["bond_label"]
        assert r["perccln"] > 0
        gval = O.f64(nb)
        O.lib().or_bond_values(rule, nb, b1, b2, bl, s, r["perccln"], 1.0, 1e-12, gval)
        sa, ija, itemp, diag, k = oracle_system(lat, m, n, 0, b1, b2, gval)
        N = t - 2 * m
        rows = np.repeat(np.arange(N), np.diff(ija[:N + 1]))
        A = sp.csr_matrix((sa[N + 1:k], (rows, ija[N + 1:k] - 1)), shape=(N, N)) + \
            sp.diags(sa[:N])
        v = spla.spsolve(A.tocsc(), itemp)
        gt, gb = C.c_double(), C.c_double()
        O.lib().or_currents(lat, m, n, 0, nb, b1, b2, gval, diag, v, 1.0, 0.0, 1, C.byref(gt),
                            C.byref(gb))
        assert rel(r["gtop"], gt.value) < 1e-9, (kind, r["gtop"], gt.value)
        assert rel(r["gbot"], gb.value) < 1e-9, (kind, r["gbot"], gb.value)


def test_multiple_spanning_clusters_use_lowest_label():
    """Hazard H4: with >1 spanning cluster only the lowest reference label
    gets g0; the GPU path resolves it with the host replay."""
    lat, m, n = 0, 24, 6  # wide and short: several spanning clusters are common
    nb = api.nbonds(lat, m, n, 0)
    found = 0
    for seed in range(1, 400):
        order = api.shuffled_ids(nb, seed)
        tb = int(0.5 * nb)
        with api.Context(lat, m, n, 0) as ctx:
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
            li = ctx.label()
            if li["nspan"] < 2:
                continue
            found += 1
            ref = api.replay_labels(lat, m, n, 0, PL.BOND, bond_order=order, nbond=tb)
            assert li["replayed"] == 1 and li["perccln"] == ref["perccln"]
            c = ctx.conductance(tol=1e-14, itmax=100000)
        b1, b2 = api.bond_list(lat, m, n, 0)
        gval = O.f64(nb)
        O.lib().or_bond_values(0, nb, b1, b2, ref["bond_label"], O.i32(1), ref["perccln"], 1.0,
                               1e-12, gval)
        oc = O.conductance(lat, m, n, 0, b1, b2, gval, tol=1e-14, itmax=100000)
        assert rel(c["gtop"], oc["gtop"]) < REL
        if found >= 3:
            break
    assert found >= 1


def test_nr_linbcg_symbol():
    """linbcg_ (F77 ABI, COMMON /mat/ via perc_nr_bind) vs the oracle's
    literal linbcg on the reference 50x50 system."""
    lat, m, n = 0, 50, 50
    b1, b2 = api.bond_list(lat, m, n, 0)
    nb = len(b1)
    order = api.shuffled_ids(nb, 626504)
    ref = api.replay_labels(lat, m, n, 0, PL.BOND, bond_order=order, nbond=int(0.6 * nb))
    gval = O.f64(nb)
    O.lib().or_bond_values(0, nb, b1, b2, ref["bond_label"], O.i32(1), ref["perccln"], 1.0, 1e-12,
                           gval)
    sa, ija, itemp, diag, k = oracle_system(lat, m, n, 0, b1, b2, gval)
    N = m * n - 2 * m
    oc = O.conductance(lat, m, n, 0, b1, b2, gval)
    L = P.lib()
    L.perc_nr_bind(sa.ctypes.data, ija.ctypes.data, len(sa))
    x = np.zeros(N)
    nn, itol, itmax, it = C.c_int(N), C.c_int(2), C.c_int(2500), C.c_int()
    tol, err = C.c_double(1e-8), C.c_double()
    b = itemp.copy()
    L.linbcg_(C.byref(nn), b.ctypes.data, x.ctypes.data, C.byref(itol), C.byref(tol),
              C.byref(itmax), C.byref(it), C.byref(err))
    assert L.perc_nr_status() == 0
    assert abs(it.value - oc["iter"]) <= 1
    assert np.max(np.abs(x - oc["vint"])) < 1e-6
    # dsprsax_ bitwise
    y, yo = np.zeros(N), O.f64(N)
    L.dsprsax_(sa.ctypes.data, ija.ctypes.data, x.ctypes.data, y.ctypes.data, C.byref(nn))
    O.lib().or_dsprsax(sa, ija, x, yo, N)
    assert np.array_equal(y.view(np.uint64), yo.view(np.uint64))
    L.perc_nr_bind(None, None, 0)


def test_bond_cond_rows_against_reference():
    for v in [v for v in G.variants() if G.meta(v)["kind"] == "bond_cond"]:
        p = G.meta(v)["params"]
        txt = G.text(v, "bondcond.txt").decode().splitlines()
        res = api.bond_cond_grid(p["lattice"], p["m"], p["n"], p["pbc"], p["seed"],
                                 p["numtrials"])
        want, cur = [], None
        for line in txt:
            if "Trial #" in line:
                cur = dict(rows=[])
                want.append(cur)
            elif cur is not None and line.count(",") == 3:
                cur["rows"].append([float(x) for x in line.split(",")])
            elif "lattice-spanning cluster:" in line:
                cur["perccln"] = int(line.split(":")[1])
            elif "pc =" in line:
                cur["pc"] = float(line.split("=")[1])
        for tr, w in zip(res, want):
            assert len(tr["rows"]) == len(w["rows"])
            for r, wr in zip(tr["rows"], w["rows"]):
                assert "%12.9f" % r["pb"] == "%12.9f" % wr[0]
                # f12.9 text: agree to the printed precision
                assert abs(r["gbot"] - wr[1]) <= 2e-9 and abs(r["gtop"] - wr[2]) <= 2e-9
            assert tr["pc"] == w["pc"]
            assert tr["perccln"] == w["perccln"]


@pytest.mark.parametrize("L_,p", [(1024, 0.6), (1024, 0.5)])
def test_full_size_properties(L_, p):
    """1024^2 (config 2 size): the reported err equals the recomputed
    residual, current is conserved at tight tolerance, labels partition."""
    nb = api.nbonds(0, L_, L_, 0)
    order = api.shuffled_ids(nb, 4562929)
    with api.Context(0, L_, L_, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        li = ctx.label()
        if li["nspan"] == 0:
            pytest.skip("no spanning cluster for this seed")
        c = ctx.conductance(tol=1e-12, itmax=10 ** 6, vint=True)
        s = ctx.system()
        N = L_ * L_ - 2 * L_
        rows = np.repeat(np.arange(N), np.diff(s["rowptr"]))
        ax = s["diag"] * c["vint"] + np.bincount(rows, weights=s["val"] * c["vint"][s["col"]],
                                                 minlength=N)
        res = np.sqrt(np.sum((s["rhs"] - ax) ** 2)) / np.sqrt(np.sum((s["rhs"] / s["diag"]) ** 2))
        # the recomputed true residual ||b - A x|| / bnrm meets the tolerance
        # the recursive residual (linbcg's err) reported
        assert c["err"] <= 1e-12 and res < 1e-11
        # current conservation up to the 1e-12 leak currents that the 1e-10
        # sprsin threshold drops from the terminal sums (hazard H5)
        assert abs(c["gtop"] - c["gbot"]) < 1e-8


def test_headline_size_properties():
    """BASELINE metric size (4096^2 bond, p = 0.6, uniform order as bench.py,
    reference settings tol 1e-8, itol 2): the default march solve and the
    LDS-tiled kernels (another q.p association) agree on the iteration
    count within 1 and on Gtop to the solver's tolerance; the recomputed
    true residual of the returned voltages meets the tolerance; the two
    terminal currents agree to the tolerance's precision."""
    L_, p = 4096, 0.6
    nb = api.nbonds(0, L_, L_, 0)
    seed = int(api.trial_seeds(58302, 1)[0])
    order = (np.random.default_rng(seed).permutation(nb)[:int(p * nb)] + 1).astype(np.int32)
    out = {}
    with api.Context(0, L_, L_, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=len(order))
        assert ctx.label()["nspan"] >= 1
        for fmt in (PL.FMT_STENCIL, PL.FMT_STENCIL_TILED):
            ctx.set_matrix_format(fmt)
            out[fmt] = ctx.conductance(tol=1e-8, itmax=10 ** 6, vint=fmt == PL.FMT_STENCIL)
            assert ctx.matrix_format() == fmt
        s = ctx.system()
    c, t = out[PL.FMT_STENCIL], out[PL.FMT_STENCIL_TILED]
    assert c["err"] <= 1e-8 and t["err"] <= 1e-8
    assert abs(c["iter"] - t["iter"]) <= 1
    assert rel(c["gtop"], t["gtop"]) < 1e-6 and rel(c["gbot"], t["gbot"]) < 1e-6
    assert rel(c["gtop"], c["gbot"]) < 1e-5
    N = L_ * L_ - 2 * L_
    rows = np.repeat(np.arange(N, dtype=np.int32), np.diff(s["rowptr"]))
    ax = s["diag"] * c["vint"] + np.bincount(rows, weights=s["val"] * c["vint"][s["col"]],
                                             minlength=N)
    res = np.sqrt(np.sum((s["rhs"] - ax) ** 2)) / np.sqrt(np.sum((s["rhs"] / s["diag"]) ** 2))
    assert res < 2e-8


def test_large_vector_grids_8192():
    """8192^2 (config 5 size; vectors past the Infinity Cache: row-major
    march, P and B on 8-row bands, the short in-order B grid): the fused
    march solve
    against the split kernels (fixed 8192-workgroup grid, another dot
    association): iteration count within 1, Gtop/Gbot to the tolerance,
    current conserved."""
    L_, p = 8192, 0.9
    nb = api.nbonds(0, L_, L_, 0)
    order = (np.random.default_rng(77).permutation(nb)[:int(p * nb)] + 1).astype(np.int32)
    out = {}
    with api.Context(0, L_, L_, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=len(order))
        assert ctx.label()["nspan"] >= 1
        for fmt in (PL.FMT_STENCIL, PL.FMT_STENCIL_SPLIT):
            ctx.set_matrix_format(fmt)
            out[fmt] = ctx.conductance(tol=1e-8, itmax=10 ** 6)
            assert ctx.matrix_format() == fmt
            if fmt == PL.FMT_STENCIL:
                info = ctx.march_info()
                assert info["band_rows"] == 8 and not info["slots"] and not info["strips"]
    c, t = out[PL.FMT_STENCIL], out[PL.FMT_STENCIL_SPLIT]
    assert c["err"] <= 1e-8 and t["err"] <= 1e-8
    assert abs(c["iter"] - t["iter"]) <= 1
    assert rel(c["gtop"], t["gtop"]) < 1e-6 and rel(c["gbot"], t["gbot"]) < 1e-6
    assert rel(c["gtop"], c["gbot"]) < 1e-5


MARCH_MODES = (PL.MARCH_DEFAULT, 0, PL.MARCH_QFREE, PL.MARCH_ALT, PL.MARCH_QFREE | PL.MARCH_ALT,
               PL.MARCH_STRIPS | PL.MARCH_QFREE, PL.MARCH_STRIPS | PL.MARCH_QFREE | PL.MARCH_ALT,
               PL.MARCH_STRIPS | PL.MARCH_QFREE | PL.MARCH_ALT | PL.MARCH_SLOTS,
               PL.MARCH_STRIPS | PL.MARCH_QFREE | PL.MARCH_ALT | PL.MARCH_TAG,
               PL.MARCH_STRIPS | PL.MARCH_QFREE | PL.MARCH_ALT | PL.MARCH_TAG | PL.MARCH_NIBBLE)


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 256, 150, 0, 0.6), (1, 128, 99, 1, 0.42),
                                           (0, 384, 40, 1, 0.55),
                                           # wide lattices, few rows
                                           (0, 1536, 40, 1, 0.55), (1, 1024, 45, 0, 0.42),
                                           (0, 2048, 21, 0, 0.6), (1, 512, 70, 1, 0.42)])
def test_march_band_heights(lat, m, n, pbc, p):
    """Register-march kernel at band heights from 1 row to more than the
    lattice (partial last band, single band), against the LDS-tiled kernel:
    same solve up to the q.p association; the x rows next to the electrodes
    and the currents come from the same per-row arithmetic."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 1234)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        ctx.set_matrix_format(PL.FMT_STENCIL_TILED)
        ref = ctx.conductance(tol=1e-12, itmax=100000, vint=True)
        assert ctx.matrix_format() == PL.FMT_STENCIL_TILED
        ctx.set_matrix_format(PL.FMT_STENCIL)
        for mode in MARCH_MODES:
            ctx.set_march_mode(mode)
            for rows in (1, 2, 3, 7, 32, 64):
                ctx.set_march_rows(rows)
                c = ctx.conductance(tol=1e-12, itmax=100000, vint=True)
                assert ctx.matrix_format() == PL.FMT_STENCIL
                assert abs(c["iter"] - ref["iter"]) <= 2, (mode, rows)
                assert rel(c["gtop"], ref["gtop"]) < REL, (mode, rows)
                assert rel(c["gbot"], ref["gbot"]) < REL, (mode, rows)
                assert np.max(np.abs(c["vint"] - ref["vint"])) < 1e-6, (mode, rows)
        ctx.set_march_rows(0)
        ctx.set_march_mode(PL.MARCH_DEFAULT)


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 256, 150, 0, 0.6), (1, 256, 99, 0, 0.42),
                                           (0, 384, 40, 1, 0.55), (1, 128, 64, 1, 0.42),
                                           (0, 1024, 50, 1, 0.55), (1, 2048, 30, 0, 0.42),
                                           # resident solve with 2048 columns (default mode)
                                           (0, 2048, 600, 0, 0.5)])
def test_march_modes_one_iteration_bitwise(lat, m, n, pbc, p):
    """Every march mode computes the same per-row numbers: with itmax = 1
    (one iteration: p = r/d, q = A p, r -= ak q, one stop test) the voltages
    agree with the split kernels up to ak's association only -- and with
    the same ak they would be bitwise; here: 1e-13 relative."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 4321)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        ctx.set_matrix_format(PL.FMT_STENCIL_SPLIT)
        ref = ctx.conductance(tol=1e-30, itmax=3, vint=True)
        ctx.set_matrix_format(PL.FMT_STENCIL)
        for mode in MARCH_MODES:
            ctx.set_march_mode(mode)
            c = ctx.conductance(tol=1e-30, itmax=3, vint=True)
            assert c["iter"] == ref["iter"]
            assert np.max(np.abs(c["vint"] - ref["vint"])) <= 1e-13 * np.max(np.abs(ref["vint"]))
            assert rel(c["err"], ref["err"]) < 1e-12
            # x on the electrode rows only (the default): bitwise the same there
            part = ctx.conductance(tol=1e-30, itmax=3)
            assert part["gtop"] == c["gtop"] and part["gbot"] == c["gbot"], mode


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 512, 512, 0, 0.6), (1, 384, 300, 0, 0.42),
                                           (0, 1024, 1024, 0, 0.55), (0, 256, 160, 1, 0.6)])
def test_tagged_reduction_is_bitwise_the_ticket_one(lat, m, n, pbc, p):
    """PERC_MARCH_TAG (tagged-granule partials, no store drain before the
    tickets): the same totals term for term as the last-arriving-workgroup
    reduction, so the whole solve -- iteration count, err history, Gtop,
    Gbot, every voltage -- is bitwise the same, at the reference tolerance
    and converged."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 2718)
    base = PL.MARCH_QFREE | PL.MARCH_ALT | PL.MARCH_STRIPS  # the march, not the resident solve
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        for tol in (1e-8, 1e-13):
            out = []
            for mode in (base, base | PL.MARCH_TAG):
                ctx.set_march_mode(mode)
                c = ctx.conductance(tol=tol, itmax=10 ** 6, vint=True)
                c["hist"] = ctx.err_history()
                info = ctx.march_info()
                assert info["kernel"] == "wave" and info["tag"] == bool(mode & PL.MARCH_TAG)
                out.append(c)
            a = out[0]
            for b in out[1:]:
                assert a["iter"] == b["iter"] and a["err"] == b["err"], (tol, a["iter"], b["iter"])
                assert np.array_equal(a["hist"].view(np.uint64), b["hist"].view(np.uint64))
                assert a["gtop"] == b["gtop"] and a["gbot"] == b["gbot"], tol
                assert np.array_equal(a["vint"].view(np.uint64), b["vint"].view(np.uint64))
        ctx.set_march_mode(PL.MARCH_DEFAULT)


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 512, 512, 0, 0.6), (1, 384, 300, 0, 0.42),
                                           (0, 1024, 1024, 0, 0.55), (0, 256, 160, 1, 0.6),
                                           (0, 128, 1400, 0, 0.6), (0, 2048, 2048, 0, 0.6)])
def test_slot_weighted_bands_solve_the_same_system(lat, m, n, pbc, p):
    """PERC_MARCH_SLOTS (one workgroup per CU and round, bands sized by the
    round): the rows are a partition of the lattice whatever the weights, so
    the solve is the static march's up to the dot products' association --
    iteration count within 2, Gtop / Gbot to the solver tolerance, the
    voltages -- for the default weights and extreme ones."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 1618)
    base = PL.MARCH_QFREE | PL.MARCH_ALT | PL.MARCH_STRIPS
    out = []
    for mode, w in ((base, None), (base | PL.MARCH_SLOTS, None), (base | PL.MARCH_SLOTS, (100, 30, 5)),
                    (base | PL.MARCH_SLOTS, (1, 1, 400))):
        with api.Context(lat, m, n, pbc) as ctx:
            if w:  # perc_set_band_weights: P and B
                ctx.set_band_weights(0, w)
                ctx.set_band_weights(1, w)
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
            if ctx.label()["nspan"] == 0:
                pytest.skip("no spanning cluster")
            ctx.set_march_mode(mode)
            out.append(ctx.conductance(tol=1e-12, itmax=200000, vint=True))
            info = ctx.march_info()
            assert info["kernel"] == "wave"
            if not mode & PL.MARCH_SLOTS:
                assert not info["slots"]
            elif (m, n) in ((1024, 1024), (2048, 2048)):
                assert info["slots"]  # (fewer rows than one round of bands: static)
    a = out[0]
    for b in out[1:]:
        assert abs(a["iter"] - b["iter"]) <= 2, (a["iter"], b["iter"])
        assert rel(b["gtop"], a["gtop"]) < REL and rel(b["gbot"], a["gbot"]) < REL
        assert np.max(np.abs(b["vint"] - a["vint"])) < 1e-6


@pytest.mark.parametrize("strips", [True, False])
@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 512, 512, 0, 0.6), (0, 256, 160, 1, 0.6),
                                           (0, 1024, 1024, 0, 0.55), (0, 128, 1400, 0, 0.6),
                                           (0, 384, 200, 1, 0.5)])
def test_nibble_codes_are_bitwise_the_u16_codes(lat, m, n, pbc, p, strips):
    """PERC_MARCH_NIBBLE (the march reads one 4-bit slot mask per site,
    count and form from the column class; strip-major, and row-major as past
    the Infinity Cache -- STRIPS off): the codes it rebuilds are the u16
    codes (k_pack_nib checks every row), so the whole solve -- iteration
    count, err history, Gtop, Gbot, every voltage -- is bitwise the u16-code
    solve's.  Row-major with pbc: both runs on the u16 codes (the nibble
    kernels there are the open square lattice's)."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 2207)
    base = PL.MARCH_DEFAULT & ~PL.SOLVE_RESIDENT  # the march, not the resident solve
    if not strips:
        base &= ~PL.MARCH_STRIPS
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        for tol in (1e-8, 1e-13):
            out = []
            for mode in (base, base & ~PL.MARCH_NIBBLE):
                ctx.set_march_mode(mode)
                c = ctx.conductance(tol=tol, itmax=10 ** 6, vint=True)
                c["hist"] = ctx.err_history()
                info = ctx.march_info()
                assert info["kernel"] == "wave" and info["strips"] == strips, info
                # (the row-major nibble kernels compile the open-square path
                # only: pbc lattices keep the u16 codes there)
                assert info["nibble"] == (bool(mode & PL.MARCH_NIBBLE) and (strips or not pbc)), info
                out.append(c)
            a, b = out
            assert a["iter"] == b["iter"] and a["err"] == b["err"], (tol, a["iter"], b["iter"])
            assert np.array_equal(a["hist"].view(np.uint64), b["hist"].view(np.uint64))
            assert a["gtop"] == b["gtop"] and a["gbot"] == b["gbot"], tol
            assert np.array_equal(a["vint"].view(np.uint64), b["vint"].view(np.uint64))
        ctx.set_march_mode(PL.MARCH_DEFAULT)


def test_table_division_is_ieee_division():
    """The solver forms z = r/d as div_tab(r, {d, RN(1/d)}) (one product and
    two fmas); bitwise IEEE division over 2^30 random pairs (a over 600
    binades and signed zeros, d = Kirchhoff diagonals and random values)."""
    out = np.zeros(3, dtype=np.uint64)
    for seed in (1, 0xC0FFEE):
        assert P.lib().perc_selftest_division(1 << 29, seed, out.ctypes.data) == 0
        assert out[0] == 0, (int(out[0]), np.array(out[1:]).view(np.float64))


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 1024, 1024, 0, 0.6), (1, 1024, 1024, 0, 0.42),
                                           (0, 1024, 40, 0, 0.6), (1, 1024, 300, 0, 0.42),
                                           (0, 1024, 700, 0, 0.55),
                                           # 2048 columns: two per thread, q formed twice
                                           (0, 2048, 2048, 0, 0.6), (0, 2048, 300, 0, 0.55),
                                           (0, 2048, 1500, 0, 0.58),
                                           (1, 2048, 800, 0, 0.42),
                                           # m < 1024: m threads per workgroup
                                           (0, 256, 256, 0, 0.6), (1, 128, 300, 0, 0.42),
                                           (0, 512, 400, 0, 0.55), (1, 512, 512, 0, 0.42),
                                           (0, 192, 300, 0, 0.6), (1, 640, 500, 0, 0.42),
                                           (0, 960, 700, 0, 0.55),
                                           # widths that are not whole waves
                                           (0, 1000, 1000, 0, 0.6), (1, 300, 301, 0, 0.42),
                                           (0, 100, 150, 0, 0.6)])
def test_resident_solve_matches_march(lat, m, n, pbc, p):
    """The persistent resident solve (one cooperative launch, p in LDS,
    two grid-wide reductions per iteration; bands of 1..4 rows per CU)
    against the launched march kernels: same per-row arithmetic, so the
    same solve up to the association of the dots."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 2024)
    out = {}
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        for mode in (PL.MARCH_ALT, PL.MARCH_DEFAULT):
            ctx.set_march_mode(mode)
            c = ctx.conductance(tol=1e-12, itmax=100000, vint=True)
            out[mode] = (c, ctx.march_info()["kernel"])
            # boundary rows only (the default): bitwise-identical to the full solve's
            part = ctx.conductance(tol=1e-12, itmax=100000)
            assert part["gtop"] == c["gtop"] and part["iter"] == c["iter"]
    (cm, km), (cr, kr) = out[PL.MARCH_ALT], out[PL.MARCH_DEFAULT]
    # (widths that are not a multiple of 128 have no march: LDS tiles)
    assert kr == "resident" and km == ("wave" if m % 128 == 0 else "none")
    assert abs(cr["iter"] - cm["iter"]) <= 2
    assert rel(cr["gtop"], cm["gtop"]) < REL and rel(cr["gbot"], cm["gbot"]) < REL
    assert np.max(np.abs(cr["vint"] - cm["vint"])) < 1e-6


@pytest.mark.parametrize("lat,m,n,p", [(0, 1024, 1024, 0.5), (1, 1024, 1024, 0.42), (0, 2048, 600, 0.55),
                                       (0, 512, 300, 0.6)])
def test_resident_grouped_and_flat_reductions(lat, m, n, p, monkeypatch):
    """The resident solve's two reduction transports (perc_resident.h):
    the XCD-grouped all-reduction (default; workgroups take their bands by
    XCD and rank) and the flat all-gather it falls back to when the
    workgroups sit unevenly on the XCDs (forced here with PERC_RES_FLAT=1):
    the same solve up to the association of the sums, and each repeatable
    bitwise (the grouped association is fixed in logical ids, whatever the
    placement).  perc_last_solve reports which transport ran: grouped where
    the grid can sit G / 8 per XCD (G = 256 at 1022 rows, 200 at 598 rows on
    256 CUs), flat from the host where it cannot (G = 149 at 298 rows) and
    under PERC_RES_FLAT."""
    nb = api.nbonds(lat, m, n, 0)
    order = api.shuffled_ids(nb, 77)
    nrows = n - 2
    H = -(-nrows // 256)  # rows per workgroup on MI355X's 256 CUs (res_geometry)
    G = -(-nrows // H)
    even = G % 8 == 0 and G // 8 <= 64  # kResXcdMax
    out = {}
    with api.Context(lat, m, n, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        for flat in ("0", "1"):
            monkeypatch.setenv("PERC_RES_FLAT", flat)
            a = ctx.conductance(tol=1e-12, itmax=200000, vint=True)
            ran = ctx.last_solve()
            assert ran["kernel"] == "resident"
            assert ran["xcd_grouped"] == (flat == "0" and even), (flat, G, ran)
            b = ctx.conductance(tol=1e-12, itmax=200000, vint=True)
            assert (a["iter"], a["gtop"], a["gbot"]) == (b["iter"], b["gtop"], b["gbot"]), flat
            assert np.array_equal(a["vint"], b["vint"]), flat
            out[flat] = a
    g, f = out["0"], out["1"]
    assert abs(g["iter"] - f["iter"]) <= 2
    assert rel(g["gtop"], f["gtop"]) < REL and rel(g["gbot"], f["gbot"]) < REL
    assert np.max(np.abs(g["vint"] - f["vint"])) < 1e-6


@pytest.mark.parametrize("kind,rule,lat,m,n,ps,pb", [(PL.BOND, PL.RULE_BOND, 0, 64, 64, 0, 0.6),
                                                     (PL.SITE, PL.RULE_SITE, 1, 48, 48, 0.6, 0),
                                                     (PL.SITEBOND, PL.RULE_MIXED, 0, 48, 40,
                                                      0.9, 0.8)])
def test_random_conductance_vs_direct_solve(kind, rule, lat, m, n, ps, pb):
    """ConductCalc.m condtype 2: spanning bonds get -g0*rand (MATLAB twister
    order: one draw per such bond in bond order).  Solved on the CSR
    operator; Gtop/Gbot against a direct sparse solve of the oracle system
    with the same values (parity with MATLAB's own draws unpinned)."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    t, nb = m * n, api.nbonds(lat, m, n, 0)
    so, bo = api.shuffled_ids(t, 31), api.shuffled_ids(nb, 32)
    ts, tb = int(ps * t), int(pb * nb)
    b1, b2 = api.bond_list(lat, m, n, 0)
    with api.Context(lat, m, n, 0) as ctx:
        ctx.occupy(kind, site_order=so if ts else None, nsites=ts,
                   bond_order=bo if tb else None, nbonds_=tb)
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        ln = ctx.label_numbers(kind)
        bl = ln["bond_label"] if ln["bond_label"] is not None else O.i32(nb)
        sl = ln["site_label"] if ln["site_label"] is not None else O.i32(t)
        w = api.conductcalc_weights(rule, b1, b2, bl, sl, ln["perccln"])
        ctx.set_bond_weights(w)
        c = ctx.conductance(rule, PL.CUR_MATLAB, tol=1e-14, itmax=400000)
        assert ctx.matrix_format() == PL.FMT_CSR
        # the same weights drawn inside libperc (the C / Fortran route): the same solve bitwise
        ctx.set_conductcalc_weights(rule)
        c_lib = ctx.conductance(rule, PL.CUR_MATLAB, tol=1e-14, itmax=400000)
        assert (c_lib["gtop"], c_lib["gbot"], c_lib["iter"]) == (c["gtop"], c["gbot"], c["iter"])
        ctx.set_bond_weights(None)
        c_fixed = ctx.conductance(rule, PL.CUR_MATLAB, tol=1e-14, itmax=400000)
    gval = O.f64(nb)
    O.lib().or_bond_values(rule, nb, b1, b2, np.ascontiguousarray(bl, np.int32),
                           np.ascontiguousarray(sl, np.int32), ln["perccln"], 1.0, 1e-12, gval)
    inc = gval == -1.0
    gval[inc] = -1.0 * w[inc]
    sa, ija, itemp, diag, k = oracle_system(lat, m, n, 0, b1, b2, gval)
    N = t - 2 * m
    rows = np.repeat(np.arange(N), np.diff(ija[:N + 1]))
    A = sp.csr_matrix((sa[N + 1:k], (rows, ija[N + 1:k] - 1)), shape=(N, N)) + sp.diags(sa[:N])
    v = spla.spsolve(A.tocsc(), itemp)
    gt, gb = C.c_double(), C.c_double()
    O.lib().or_currents(lat, m, n, 0, nb, b1, b2, gval, diag, v, 1.0, 0.0, 1, C.byref(gt),
                        C.byref(gb))
    assert rel(c["gtop"], gt.value) < 1e-9 and rel(c["gbot"], gb.value) < 1e-9
    assert rel(c["gtop"], c_fixed["gtop"]) > 1e-3  # the weights did act


# ------------------------------------------------------------ edge cases
@pytest.mark.parametrize("kind,lat,pbc", [(PL.BOND, 0, 0), (PL.SITE, 1, 1), (PL.SITEBOND, 0, 1)])
def test_empty_occupancy_is_not_spanning(kind, lat, pbc):
    """Nothing occupied: no cluster spans, the conductance is G = 0 with
    status 1 (bond_cond.f:484-487), no solve runs."""
    m = n = 64
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(kind, site_order=np.zeros(1, np.int32), nsites=0,
                   bond_order=np.zeros(1, np.int32), nbonds_=0)
        li = ctx.label()
        assert li["nspan"] == 0
        c = ctx.conductance(PL.RULE_BOND if kind == PL.BOND else PL.RULE_MIXED)
        assert c["status"] == 1 and c["gtop"] == 0.0 and c["iter"] == 0


@pytest.mark.parametrize("m,n,pbc", [(1024, 1024, 0), (1024, 1024, 1), (2048, 512, 0),
                                     (256, 2000, 1)])
def test_full_square_lattice_analytic(m, n, pbc):
    """Every bond occupied (a maximum-size cluster): each row is an
    equipotential, so G = m / (n - 1) exactly (horizontal bonds carry no
    current); resident, march and pbc paths alike."""
    nb = api.nbonds(0, m, n, pbc)
    with api.Context(0, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=np.arange(1, nb + 1, dtype=np.int32), nbonds_=nb)
        li = ctx.label()
        assert li["nspan"] == 1
        c = ctx.conductance(tol=1e-13, itmax=10 ** 6)
    want = m / (n - 1)
    assert rel(c["gtop"], want) < 1e-9 and rel(c["gbot"], want) < 1e-9


@pytest.mark.parametrize("lat,m,n,pbc", [(1, 64, 64, 0), (1, 64, 64, 1), (0, 3, 3, 0),
                                         (0, 3, 4, 0), (1, 4, 4, 0), (0, 4, 3, 1)])
def test_full_and_tiny_lattices_vs_oracle(lat, m, n, pbc):
    """Fully occupied triangular lattices and the smallest lattices libperc
    takes (m, n >= 3, even m on the triangular lattice: one or two interior
    rows, 3-4 columns): GPU solve vs
    the oracle's literal linbcg on the same system."""
    b1, b2 = api.bond_list(lat, m, n, pbc)
    nb = len(b1)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=np.arange(1, nb + 1, dtype=np.int32), nbonds_=nb)
        assert ctx.label()["nspan"] == 1
        c = ctx.conductance(tol=1e-14, itmax=100000)
    oc = O.conductance(lat, m, n, pbc, b1, b2, -np.ones(nb), tol=1e-14, itmax=100000)
    assert rel(c["gtop"], oc["gtop"]) < REL and rel(c["gbot"], oc["gbot"]) < REL
    assert abs(c["iter"] - oc["iter"]) <= 1


@pytest.mark.parametrize("lat,m,n,pbc,p", [(0, 90, 90, 0, 0.6), (1, 64, 80, 1, 0.42),
                                           (0, 100, 80, 1, 0.55), (1, 50, 50, 0, 0.4)])
def test_small_solver_matches_launched(lat, m, n, pbc, p):
    """The one-workgroup solve (k_cg_small, default format, N <= 8192)
    against the launched kernels of an explicit format: same per-row
    arithmetic, dots associated differently -- iterations +-1 and Gtop /
    Gbot / voltages to 1e-10 at tol 1e-13; and it is the solver that ran."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, 999 + m)
    out = {}
    for fmt in (PL.FMT_AUTO, PL.FMT_STENCIL_SPLIT, PL.FMT_CSR):
        with api.Context(lat, m, n, pbc) as ctx:
            ctx.set_matrix_format(fmt)
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
            if ctx.label()["nspan"] == 0:
                pytest.skip("no spanning cluster")
            out[fmt] = ctx.conductance(tol=1e-13, itmax=100000, vint=True)
            assert (ctx.march_info()["kernel"] == "small") == (fmt == PL.FMT_AUTO)
    s = out[PL.FMT_AUTO]
    for fmt in (PL.FMT_STENCIL_SPLIT, PL.FMT_CSR):
        c = out[fmt]
        assert abs(s["iter"] - c["iter"]) <= 1
        assert rel(s["gtop"], c["gtop"]) < REL and rel(s["gbot"], c["gbot"]) < REL
        assert np.max(np.abs(s["vint"] - c["vint"])) < 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("kind,rule,m,n,pbc", [(PL.BOND, PL.RULE_BOND, 256, 150, 0),
                                               (PL.BOND, PL.RULE_BOND, 131, 90, 1),
                                               (PL.SITEBOND, PL.RULE_MIXED, 200, 64, 0),
                                               (PL.SITEBOND, PL.RULE_MIXED, 96, 70, 1),
                                               (PL.SITE, PL.RULE_SITE, 130, 70, 1)])
def test_closed_form_assembly_is_the_general_one(kind, rule, m, n, pbc, monkeypatch):
    """k_assemble's closed-form paths for the square lattice (interior,
    column 0, column m-1; with and without pbc) write what its general path (PERC_ASM_GENERIC=1: nearestn +
    bond_id per neighbour) writes: the same CSR system bitwise and the same
    solve."""
    nb, t = api.nbonds(0, m, n, pbc), m * n
    out = []
    for generic in ("0", "1"):
        monkeypatch.setenv("PERC_ASM_GENERIC", generic)
        with api.Context(0, m, n, pbc) as ctx:
            ctx.occupy_random(kind, int(0.9 * t) if kind != PL.BOND else 0, int(0.62 * nb), 4242)
            assert ctx.label()["nspan"] >= 1
            c = ctx.conductance(rule=rule, itmax=25)
            sysm = ctx.system()
        out.append((c, sysm))
    (c0, s0), (c1, s1) = out
    for key in ("rowptr", "col"):
        assert np.array_equal(s0[key], s1[key])
    for key in ("val", "diag", "rhs"):
        assert np.array_equal(s0[key].view(np.uint64), s1[key].view(np.uint64)), key
    assert (c0["gtop"], c0["gbot"], c0["iter"]) == (c1["gtop"], c1["gbot"], c1["iter"])


