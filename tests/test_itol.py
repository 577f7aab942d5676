"""linbcg's other stopping rules, itol 3 and 4 (Square/bondc.f:771-775,
816-832): NR's step-size estimate |z| / |z(k-1) - z| * |ak| |p| / |x| with
snrm in the L2 (itol 3) or max (itol 4) norm, and its two `goto 100`
branches that iterate on without the tolerance test.

The reference's drivers only call itol 2, so no reference output pins
these modes ("parity unpinned" against the reference itself): the oracle's
or_linbcg restates bondc.f:750-838 for every itol and is checked here
against a dense solve; the device solve (perc_conductance / linbcg_ with
itol 3 or 4: dev_solve_x34) is checked against that oracle -- bitwise in
the literal dot order (iteration count, the err history, Gtop, Gbot, every
voltage), to a tolerance in the fast order.
"""
import numpy as np
import pytest

import oracle_lib as O
from percolation_amd import _lib as PL
from percolation_amd import api

CASES = [(0, 64, 64, 0, 0.6, 21), (1, 64, 50, 0, 0.42, 22), (0, 96, 80, 1, 0.6, 23)]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def system(lat, m, n, pbc, p, seed):
    b1, b2 = api.bond_list(lat, m, n, pbc)
    nb = len(b1)
    order = api.shuffled_ids(nb, seed)
    tb = int(p * nb)
    ref = api.replay_labels(lat, m, n, pbc, PL.BOND, bond_order=order, nbond=tb)
    assert ref["perccln"] > 0
    gval = O.f64(nb)
    O.lib().or_bond_values(0, nb, b1, b2, ref["bond_label"], O.i32(1), ref["perccln"], 1.0, 1e-12,
                           gval)
    return b1, b2, gval, order, tb


def dense(sa, ija, N):
    a = np.zeros((N, N))
    a[np.arange(N), np.arange(N)] = sa[:N]
    for i in range(N):
        for k in range(ija[i] - 1, ija[i + 1] - 1):
            a[i, ija[k] - 1] = sa[k]
    return a


@pytest.mark.parametrize("itol", [3, 4])
def test_oracle_itol34_converges_to_the_dense_solve(itol):
    lat, m, n, pbc, p, seed = 0, 24, 20, 0, 0.62, 5
    b1, b2, gval, _, _ = system(lat, m, n, pbc, p, seed)
    ref = O.conductance(lat, m, n, pbc, b1, b2, gval, itol=2, tol=1e-14, itmax=100000)
    for tol, want in ((1e-6, 1e-4), (1e-12, 1e-9)):
        oc = O.conductance(lat, m, n, pbc, b1, b2, gval, itol=itol, tol=tol, itmax=100000)
        N = len(oc["itemp"])
        x = np.linalg.solve(dense(oc["sa"], oc["ija"], N), oc["itemp"])
        assert np.max(np.abs(oc["vint"] - x)) <= want * np.max(np.abs(x)), (itol, tol)
        assert oc["err"] <= tol and oc["iter"] < 100000
        assert abs(oc["gtop"] - ref["gtop"]) <= want * abs(ref["gtop"])
    # the estimate stops later at a tighter tolerance
    lo = O.conductance(lat, m, n, pbc, b1, b2, gval, itol=itol, tol=1e-6, itmax=100000)
    hi = O.conductance(lat, m, n, pbc, b1, b2, gval, itol=itol, tol=1e-12, itmax=100000)
    assert lo["iter"] < hi["iter"]


@pytest.mark.gpu
@pytest.mark.parametrize("itol", [3, 4])
@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES)
def test_itol34_literal_is_the_oracle_bitwise(lat, m, n, pbc, p, seed, itol):
    b1, b2, gval, order, tb = system(lat, m, n, pbc, p, seed)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        for tol in (1e-8, 1e-12):
            oc = O.conductance(lat, m, n, pbc, b1, b2, gval, itol=itol, tol=tol, itmax=100000)
            ctx.set_dot_order(PL.DOT_LITERAL)
            c = ctx.conductance(itol=itol, tol=tol, itmax=100000, vint=True)
            hist = ctx.err_history()
            assert ctx.last_solve()["kernel"] == "other"
            assert c["iter"] == oc["iter"], (tol, c["iter"], oc["iter"])
            assert np.array_equal(bits(hist), bits(oc["errs"])), tol
            assert c["gtop"] == oc["gtop"] and c["gbot"] == oc["gbot"], tol
            assert np.array_equal(bits(c["vint"]), bits(oc["vint"])), tol
            # the fast order: block-partial sums, the same iterates to
            # rounding; the step-size estimate is noisy on a stagnating
            # tail, so the stop may move by a few iterations (measured: 596
            # vs 600 on the triangular case at 1e-8)
            ctx.set_dot_order(PL.DOT_FAST)
            f = ctx.conductance(itol=itol, tol=tol, itmax=100000)
            assert abs(f["iter"] - oc["iter"]) <= max(2, oc["iter"] // 50), (f["iter"], oc["iter"])
            assert abs(f["gtop"] - oc["gtop"]) <= 1e-6 * abs(oc["gtop"])


@pytest.mark.gpu
def test_illegal_itol_is_perc_eitol():
    lat, m, n = 0, 32, 32
    nb = api.nbonds(lat, m, n, 0)
    with api.Context(lat, m, n, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=api.shuffled_ids(nb, 3), nbonds_=int(0.7 * nb))
        assert ctx.label()["nspan"] > 0
        for itol in (0, 5):
            with pytest.raises(PL.PercError, match="EITOL"):
                ctx.conductance(itol=itol, tol=1e-8, itmax=1000)


@pytest.mark.gpu
@pytest.mark.parametrize("itol", [3, 4])
def test_nr_linbcg_symbol_itol34(itol):
    """linbcg_ (the NR drop-in, literal dot order by default) with itol 3 /
    4 on the reference's 50x50 system: bitwise the oracle's linbcg"""
    import ctypes as C
    import percolation_amd as P
    lat, m, n = 0, 50, 50
    b1, b2, gval, _, _ = system(lat, m, n, 0, 0.6, 626504)
    oc = O.conductance(lat, m, n, 0, b1, b2, gval, itol=itol, tol=1e-10, itmax=2500)
    sa, ija = oc["sa"].copy(), oc["ija"].copy()
    N = m * n - 2 * m
    L = P.lib()
    L.perc_nr_bind(sa.ctypes.data, ija.ctypes.data, len(sa))
    try:
        x = np.zeros(N)
        nn, it_, itmax, it = C.c_int(N), C.c_int(itol), C.c_int(2500), C.c_int()
        tol, err = C.c_double(1e-10), C.c_double()
        b = oc["itemp"].copy()
        L.linbcg_(C.byref(nn), b.ctypes.data, x.ctypes.data, C.byref(it_), C.byref(tol),
                  C.byref(itmax), C.byref(it), C.byref(err))
        assert L.perc_nr_status() == 0
        assert it.value == oc["iter"] and err.value == oc["err"], (it.value, oc["iter"])
        assert np.array_equal(bits(x), bits(oc["vint"]))
    finally:
        L.perc_nr_bind(None, None, 0)
