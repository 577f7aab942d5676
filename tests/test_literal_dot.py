"""The literal dot order on the GPU (perc_set_dot_order(h, PERC_DOT_LITERAL)).

linbcg sums its three dot products term after term in ascending j --
bknum (Square/bondc.f:785-787), akden (:803-805), snrm's sum of squares
(:872-875, bnrm :768-770).  Every other operation of an iteration is
already the reference's on the GPU (per-row bitwise: test_gpu_parity.py's
assembly / SpMV / march-mode tests), so with the sums folded in that order
the whole solve must be the reference solver's BITWISE: iteration count,
the per-iteration err history (`write (*,*) iter, err`, :834), every
interior voltage, Gtop and Gbot.  That pins the remaining difference of the
default solve to the association of the three sums alone.

Pins: every reference bondc golden (tests/golden/*bondc*, made by the
compiled reference, square / triangular / pbc / tight tolerance) in every
solver family (one-workgroup, the resident solve, LDS-tiled, split stencil,
CSR), and the oracle's literal linbcg (oracle/perc_oracle.c, itself bitwise
the reference at <= 64^2) at 128^2 .. 512^2 through the PRODUCTION kernels:
the resident cooperative solve (k_cg_res, configs 2-4's solver), the
q-free strip-major march with nibble codes and tagged reductions (k_cg_march
P / B, the metric's kernels) and the q-free ROW-MAJOR march (P on u16 codes,
B on nibble codes: the production solver wherever a vector exceeds 256 MB,
i.e. L > 4096 -- config 5's companion; forced here at 512^2 by clearing
PERC_MARCH_STRIPS), bond and ConductCalc mixed-rule systems.  Those kernels
store their rows' dot terms and the folds sum them (perc_last_solve:
lit_terms); the q-storing march is no longer part of the literal path.
"""
import numpy as np
import pytest

import golden_io as G
import oracle_lib as O
from percolation_amd import _lib as PL
from percolation_amd import api

pytestmark = pytest.mark.gpu

BONDC = [v for v in G.variants() if G.meta(v)["kind"] == "bondc" and G.meta(v)["perccln"]]
# PERC_FMT_AUTO runs the one-workgroup solver at these sizes (k_cg_small<LIT>),
# PERC_FMT_STENCIL the resident solve (k_cg_res<..., LIT>)
FAMILIES = [PL.FMT_AUTO, PL.FMT_STENCIL, PL.FMT_STENCIL_TILED, PL.FMT_STENCIL_SPLIT, PL.FMT_CSR]
# the march without the resident solve (PERC_SOLVE_RESIDENT off)
MARCH_ONLY = PL.MARCH_DEFAULT & ~PL.SOLVE_RESIDENT


# the oracle's solves, shared by the solver parametrisations of one system
# (a 512^2 literal linbcg to 1e-13 takes ~25 s of CPU: computed once)
_ORACLE = {}


def oracle_conductance(key, *args, **kw):
    if key not in _ORACLE:
        _ORACLE[key] = O.conductance(*args, **kw)
    return _ORACLE[key]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


@pytest.mark.parametrize("fmt", FAMILIES)
@pytest.mark.parametrize("v", BONDC)
def test_literal_solve_is_the_reference_bitwise(v, fmt):
    md = G.meta(v)
    p = md["params"]
    tol, itmax = p.get("tol", 1e-8), p.get("itmax", 2500)
    with api.Context(p["lattice"], p["m"], p["n"], p["pbc"]) as ctx:
        ctx.set_dot_order(PL.DOT_LITERAL)
        ctx.set_matrix_format(fmt)
        try:
            r = api.bondc(p["lattice"], p["m"], p["n"], p["pbc"], p["pb"], p["seed"], tol=tol,
                          itmax=itmax, ctx=ctx)
        except PL.PercError as e:  # this lattice has no such operator (e.g. odd m, tiles)
            pytest.skip(str(e))
        hist = ctx.err_history()
        ran = ctx.last_solve()
        c = ctx.conductance(tol=tol, itmax=itmax, vint=True)
    if fmt == PL.FMT_STENCIL and not p["pbc"]:
        # the production resident kernel, folding its own terms (pbc: wrapped
        # forms, no resident grid: the LDS-tiled kernel at m = 50)
        assert ran["kernel"] == "resident" and ran["lit_terms"], ran
    assert ran["literal"] and ran["iter"] == r["iter"], ran
    assert r["perccln"] == md["perccln"]
    assert r["iter"] == md["iter"], (r["iter"], md["iter"])
    assert np.array_equal(bits(hist), bits(md["linbcg_err"]))
    assert r["gtop"] == md["gtop"] and r["gbot"] == md["gbot"], (r["gtop"], r["gbot"])
    assert (c["gtop"], c["gbot"], c["iter"]) == (r["gtop"], r["gbot"], r["iter"])
    if "vint" in md:
        assert np.array_equal(bits(c["vint"]), bits(md["vint"]))


SOLVERS = ["resident", "march", "march_rowmajor", "csr"]
# the row-major q-free march (MARCH_STRIPS off: what runs past the Infinity
# Cache, L > 4096), with the sums folded by the host (PERC_DOT_LITERAL_HOST,
# bitwise the device fold: test_host_fold_is_the_device_fold_bitwise)
MARCH_ROWMAJOR = MARCH_ONLY & ~PL.MARCH_STRIPS
LATTICES = [(0, 128, 128, 0, 0.6, 21), (0, 256, 150, 0, 0.55, 31), (1, 128, 99, 0, 0.4, 22),
            (0, 256, 256, 1, 0.6, 32), (0, 512, 512, 0, 0.6, 33)]


@pytest.mark.parametrize("solver", SOLVERS)
@pytest.mark.parametrize("lat,m,n,pbc,p,seed", LATTICES)
def test_literal_solve_is_the_oracle_linbcg_bitwise(lat, m, n, pbc, p, seed, solver):
    """Larger lattices, m a multiple of 128, against the oracle's literal
    linbcg at the reference tolerance and at 1e-13: iter, err history, Gtop,
    Gbot and every voltage bitwise -- through the production kernels: the
    resident solve (PERC_FMT_AUTO, where the lattice fits it) and the q-free
    strip-major march (P / B, nibble codes on the square lattice, tagged
    reductions: the metric's kernels), each storing its own dot terms; and
    CSR (terms folded from q, p, r)."""
    b1, b2 = api.bond_list(lat, m, n, pbc)
    nb = len(b1)
    order = api.shuffled_ids(nb, seed)
    tb = int(p * nb)
    ref = api.replay_labels(lat, m, n, pbc, PL.BOND, bond_order=order, nbond=tb)
    assert ref["perccln"] > 0
    gval = O.f64(nb)
    O.lib().or_bond_values(0, nb, b1, b2, ref["bond_label"], O.i32(1), ref["perccln"], 1.0, 1e-12,
                           gval)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.set_dot_order(PL.DOT_LITERAL)
        if solver == "csr":
            ctx.set_matrix_format(PL.FMT_CSR)
        elif solver == "march":
            ctx.set_march_mode(MARCH_ONLY)
        elif solver == "march_rowmajor":
            ctx.set_march_mode(MARCH_ROWMAJOR)
            ctx.set_dot_order(PL.DOT_LITERAL_HOST)
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        for tol in (1e-8, 1e-13):
            oc = oracle_conductance(("bond", lat, m, n, pbc, p, seed, tol), lat, m, n, pbc, b1, b2, gval,
                                    tol=tol, itmax=100000)
            c = ctx.conductance(tol=tol, itmax=100000, vint=True)
            hist = ctx.err_history()
            ran = ctx.last_solve()
            assert ran["literal"] and ran["iter"] == c["iter"], ran
            if solver == "resident" and not pbc:  # (pbc: wrapped forms, no resident grid)
                assert ran["kernel"] == "resident" and ran["lit_terms"], ran
            elif solver == "march_rowmajor":
                # the L > 4096 production march: q-free, row-major, host folds
                # of the kernels' own terms; nibble codes (B) on the open square lattice
                assert ran["kernel"] == "march" and ran["lit_terms"] and ran["host_fold"], ran
                assert ran["qfree"] and not ran["strips"], ran
                if lat == 0 and not pbc:
                    assert ran["nibble"], ran
            elif solver != "csr":
                # the metric's kernels: q-free, strip-major, tagged; nibble
                # codes on the open square lattice
                assert ran["kernel"] == "march" and ran["lit_terms"], ran
                assert ran["qfree"] and ran["strips"] and ran["tag"], ran
                if lat == 0 and not pbc:
                    assert ran["nibble"], ran
            else:
                assert ran["kernel"] == "other" and not ran["lit_terms"], ran
            assert c["iter"] == oc["iter"], (tol, c["iter"], oc["iter"])
            assert np.array_equal(bits(hist), bits(oc["errs"])), tol
            assert c["gtop"] == oc["gtop"] and c["gbot"] == oc["gbot"], (tol, c["gtop"], oc["gtop"])
            assert np.array_equal(bits(c["vint"]), bits(oc["vint"])), tol


def mixed_system(L_, ps, pb, sseed, bseed):
    """sitebond.f's mixed occupation (reference shuffles: sites with sseed,
    bonds with bseed) labelled by the oracle's replay, its spanning cluster
    (site.f:309-344 rule with 2L-1, as make_config_golden.py) and
    ConductCalc.m's mixed-rule bond values (:134-160); None if nothing spans"""
    lib = O.lib()
    t = L_ * L_
    b1, b2, o1, o2 = O.bond_order(0, L_, L_, 0, bseed)
    nb = len(b1)
    so = O.site_order(t, sseed)
    ts, tb = int(ps * t), int(pb * nb)
    s, bl, csize, cln, _, _ = O.label_sitebond(0, L_, L_, 0, b1, b2, so, ts, o1, o2, tb, literal=False)
    perccln = lib.or_span_sites(L_, L_, s, csize, cln, 2 * L_ - 1)
    if perccln <= 0:
        return None
    gval = O.f64(nb)
    lib.or_bond_values(2, nb, b1, b2, bl, s, perccln, 1.0, 1e-12, gval)
    occ = dict(kind=PL.SITEBOND, site_order=api.shuffled_ids(t, sseed), nsites=ts,
               bond_order=api.shuffled_ids(nb, bseed), nbonds_=tb)
    return b1, b2, gval, occ


@pytest.mark.parametrize("solver", ["march", "march_rowmajor"])
def test_literal_mixed_rule_is_the_oracle_linbcg_bitwise(solver):
    """Config 5's system class (square mixed site-then-bond, ConductCalc.m
    mixed rule and currents, sitebond.f's seeds) at 512^2, ps = pb = 0.85,
    through the strip-major march (the c5m fixture's solver) and the
    ROW-MAJOR march (P on u16 codes, B on nibble codes: config 5's companion
    solver at 8192^2): iter, err history, Gtop, Gbot and every voltage
    bitwise the oracle's literal linbcg (Square/bondc.f:750-838)"""
    L_ = 512
    sysm = mixed_system(L_, 0.85, 0.85, 143285, 43716)
    assert sysm is not None, "the 512^2 mixed case must span"
    b1, b2, gval, occ = sysm
    with api.Context(0, L_, L_, 0) as ctx:
        if solver == "march":
            ctx.set_march_mode(MARCH_ONLY)
            ctx.set_dot_order(PL.DOT_LITERAL)
        else:
            ctx.set_march_mode(MARCH_ROWMAJOR)
            ctx.set_dot_order(PL.DOT_LITERAL_HOST)
        ctx.occupy(**occ)
        assert ctx.label()["nspan"] > 0
        for tol in (1e-8, 1e-13):
            oc = oracle_conductance(("mixed", L_, tol), 0, L_, L_, 0, b1, b2, gval, tol=tol, itmax=100000,
                                    rhs_rule=0, cur_rule=1, cur_thresh=0.0)
            c = ctx.conductance(PL.RULE_MIXED, PL.CUR_MATLAB, tol=tol, itmax=100000, vint=True)
            hist = ctx.err_history()
            ran = ctx.last_solve()
            assert ran["kernel"] == "march" and ran["literal"] and ran["lit_terms"], ran
            assert ran["qfree"] and ran["nibble"] and ran["strips"] == (solver == "march"), ran
            assert c["iter"] == oc["iter"], (tol, c["iter"], oc["iter"])
            assert np.array_equal(bits(hist), bits(oc["errs"])), tol
            assert c["gtop"] == oc["gtop"] and c["gbot"] == oc["gbot"], (tol, c["gtop"], oc["gtop"])
            assert np.array_equal(bits(c["vint"]), bits(oc["vint"])), tol


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", [(0, 512, 512, 0, 0.6, 33), (1, 256, 200, 0, 0.42, 7)])
def test_host_fold_is_the_device_fold_bitwise(lat, m, n, pbc, p, seed):
    """PERC_DOT_LITERAL_HOST (the serial sums on the host CPU from the terms
    the march kernels stored) against PERC_DOT_LITERAL with the same march
    (the sums folded by one GPU wave): the same IEEE adds in the same order,
    so iter, the err history, Gtop, Gbot and every voltage are identical"""
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, seed)
    out = {}
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.set_march_mode(MARCH_ONLY)
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        assert ctx.label()["nspan"] > 0
        for order_ in (PL.DOT_LITERAL, PL.DOT_LITERAL_HOST):
            ctx.set_dot_order(order_)
            c = ctx.conductance(tol=1e-10, itmax=100000, vint=True)
            out[order_] = (c, ctx.err_history(), ctx.last_solve())
    (cd, hd, rd), (ch, hh, rh) = out[PL.DOT_LITERAL], out[PL.DOT_LITERAL_HOST]
    assert rd["lit_terms"] and not rd["host_fold"] and rh["lit_terms"] and rh["host_fold"], (rd, rh)
    assert rh["kernel"] == "march" and rh["qfree"] and rh["strips"], rh
    assert (cd["iter"], cd["gtop"], cd["gbot"], cd["err"]) == (ch["iter"], ch["gtop"], ch["gbot"], ch["err"])
    assert np.array_equal(bits(hd), bits(hh))
    assert np.array_equal(bits(cd["vint"]), bits(ch["vint"]))


def test_literal_and_fast_orders_differ_by_association_only():
    """The same system in both orders at a converged tolerance: the same
    answer to 1e-10 (only the three sums' association differs), and the
    fast order comes back when asked for."""
    lat, m, n, pbc, p, seed = 0, 256, 200, 0, 0.6, 41
    nb = api.nbonds(lat, m, n, pbc)
    order = api.shuffled_ids(nb, seed)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(p * nb))
        ctx.label()
        fast = ctx.conductance(tol=1e-14, itmax=100000)
        ctx.set_dot_order(PL.DOT_LITERAL)
        lit = ctx.conductance(tol=1e-14, itmax=100000)
        ctx.set_dot_order(PL.DOT_FAST)
        again = ctx.conductance(tol=1e-14, itmax=100000)
    assert abs(lit["gtop"] - fast["gtop"]) < 1e-10 * fast["gtop"]
    assert abs(lit["gbot"] - fast["gbot"]) < 1e-10 * fast["gbot"]
    assert (again["gtop"], again["gbot"], again["iter"]) == (fast["gtop"], fast["gbot"], fast["iter"])


def test_literal_order_needs_one_slab():
    lat, m, n = 0, 256, 64
    nb = api.nbonds(lat, m, n, 0)
    with api.Context(lat, m, n, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=api.shuffled_ids(nb, 5), nbonds_=int(0.65 * nb))
        ctx.label()
        ctx.set_dot_order(PL.DOT_LITERAL)
        ctx.set_slabs(2)
        with pytest.raises(PL.PercError):
            ctx.conductance(tol=1e-8, itmax=10000)
