"""Row-slab decomposition of one CG solve (perc_set_slabs; SURVEY.md §8(f)
row 2, the linbcg loop of Square/bondc.f:780-836).

K slabs with private vectors and ghost rows, halo copies of r and slab-order
combination of the dot partials, on one device.  Per-row arithmetic is the
single-slab solve's; the iterates differ only through the association of
the dot products.  Bars: iteration count within +-1 of the single-slab
solve, Gtop/Gbot within 1e-10 relative at tol 1e-13 (and against the
oracle's literal linbcg, which is bitwise the reference at <= 64^2), and
one iteration agreeing to 1e-13 (only ak's association differs).
"""
import numpy as np
import pytest

import oracle_lib as O
from percolation_amd import _lib as PL
from percolation_amd import api

pytestmark = pytest.mark.gpu
REL = 1e-10


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def solve(lat, m, n, pbc, order, tb, nslab, **kw):
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        if ctx.label()["nspan"] == 0:
            return None
        ctx.set_slabs(nslab)
        c = ctx.conductance(**kw)
        assert ctx.matrix_format() == PL.FMT_STENCIL
        return c


CASES = [(0, 256, 200, 0, 0.6, 11), (1, 256, 150, 0, 0.45, 12), (0, 384, 120, 1, 0.58, 13),
         (1, 128, 97, 1, 0.42, 14)]


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES)
def test_slabs_match_single_slab_converged(lat, m, n, pbc, p, seed):
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, seed)
    tb = int(p * nb)
    ref = solve(lat, m, n, pbc, order, tb, 1, tol=1e-13, itmax=200000, vint=True)
    if ref is None:
        pytest.skip("no spanning cluster")
    for K in (2, 3, 4, 7):
        c = solve(lat, m, n, pbc, order, tb, K, tol=1e-13, itmax=200000, vint=True)
        assert abs(c["iter"] - ref["iter"]) <= 1, (K, c["iter"], ref["iter"])
        assert rel(c["gtop"], ref["gtop"]) < REL, (K, c["gtop"], ref["gtop"])
        assert rel(c["gbot"], ref["gbot"]) < REL, (K, c["gbot"], ref["gbot"])
        assert np.max(np.abs(c["vint"] - ref["vint"])) < 1e-8, K


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES[:2])
def test_slabs_boundary_rows_only(lat, m, n, pbc, p, seed):
    """Without vint the slabs carry x on the electrode-adjacent rows only
    (slab 0's first row, slab K-1's last row): the currents are those of
    the full-voltage slab solve, bitwise."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, seed)
    tb = int(p * nb)
    for K in (2, 5):
        full = solve(lat, m, n, pbc, order, tb, K, tol=1e-12, itmax=200000, vint=True)
        if full is None:
            pytest.skip("no spanning cluster")
        edge = solve(lat, m, n, pbc, order, tb, K, tol=1e-12, itmax=200000)
        assert edge["iter"] == full["iter"]
        assert edge["gtop"] == full["gtop"] and edge["gbot"] == full["gbot"]


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES[:3])
def test_slabs_one_iteration(lat, m, n, pbc, p, seed):
    """One iteration (p = r/d, q = A p, r -= ak q): the slab and single-slab
    voltages agree to 1e-13 relative (ak associated per slab)."""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, seed)
    tb = int(p * nb)
    ref = solve(lat, m, n, pbc, order, tb, 1, tol=1e-30, itmax=1, vint=True)
    if ref is None:
        pytest.skip("no spanning cluster")
    for K in (2, 4):
        c = solve(lat, m, n, pbc, order, tb, K, tol=1e-30, itmax=1, vint=True)
        assert c["iter"] == ref["iter"]
        scale = np.max(np.abs(ref["vint"]))
        assert np.max(np.abs(c["vint"] - ref["vint"])) <= 1e-13 * scale, K


@pytest.mark.parametrize("lat,m,n,p,seed", [(0, 128, 128, 0.6, 21), (1, 128, 100, 0.4, 22)])
def test_slabs_vs_oracle_linbcg(lat, m, n, p, seed):
    """Against the oracle's literal linbcg (CPU): reference settings (tol
    1e-8) iteration count +-1 and Gtop to the solver tolerance; converged
    (tol 1e-13) Gtop and Gbot within 1e-10."""
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
    for K in (2, 4):
        c = solve(lat, m, n, 0, order, tb, K, itmax=100000)
        ct = solve(lat, m, n, 0, order, tb, K, tol=1e-13, itmax=100000)
        assert abs(c["iter"] - oc["iter"]) <= 1, (K, c["iter"], oc["iter"])
        assert rel(c["gtop"], oc["gtop"]) < 1e-8
        assert abs(ct["iter"] - ot["iter"]) <= 1
        assert rel(ct["gtop"], ot["gtop"]) < REL and rel(ct["gbot"], ot["gbot"]) < REL


def test_slabs_at_1024():
    """1024^2 square bond at p = 0.6 (BASELINE config 2's size), K = 2 and 4
    against one slab with the same launched kernels (the resident solve is
    another association): iterations +-1 at tol 1e-12 (at 1e-13 the tail
    sits at the fp64 floor, where each association stops within a few
    iterations of the others), Gtop / Gbot within 1e-10 at tol 1e-13."""
    L_, p = 1024, 0.6
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(p * nb)
    order = (np.random.default_rng(31).permutation(nb)[:tb] + 1).astype(np.int32)

    def run(K, tol):
        with api.Context(0, L_, L_, 0) as ctx:
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
            assert ctx.label()["nspan"] > 0
            ctx.set_march_mode(PL.MARCH_ALT)  # launched march kernels
            ctx.set_slabs(K)
            return ctx.conductance(tol=tol, itmax=10 ** 6)

    ref12, ref13 = run(1, 1e-12), run(1, 1e-13)
    for K in (2, 4):
        c12, c13 = run(K, 1e-12), run(K, 1e-13)
        assert abs(c12["iter"] - ref12["iter"]) <= 1, (K, c12["iter"], ref12["iter"])
        assert abs(c13["iter"] - ref13["iter"]) <= 3, (K, c13["iter"], ref13["iter"])
        assert rel(c13["gtop"], ref13["gtop"]) < REL and rel(c13["gbot"], ref13["gbot"]) < REL


def test_slabs_need_the_march_format():
    """The slab engine runs the register-march kernels: another operator
    format is refused loudly, not silently solved another way."""
    lat, m, n, p = 0, 256, 64, 0.6
    nb = api.nbonds(lat, m, n, 0)
    order = api.shuffled_ids(nb, 5)
    with api.Context(lat, m, n, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        if ctx.label()["nspan"] == 0:
            pytest.skip("no spanning cluster")
        ctx.set_slabs(2)
        ctx.set_matrix_format(PL.FMT_CSR)
        with pytest.raises(PL.PercError):
            ctx.conductance(tol=1e-10, itmax=10000)
