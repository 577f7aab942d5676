"""GPU against the oracle at the BASELINE config sizes, through committed
fixtures (tests/golden/configs/*.json, made by
tests/golden/make_config_golden.py from oracle/perc_oracle.c: the O(N alpha)
replay labels and the literal linbcg, Square/bondc.f:189-595, on the CPU in
this container; the oracle is pinned bit-exact to the reference's own
outputs at <= 64^2 by tests/test_oracle_golden.py).

Per fixture: the occupation order is rebuilt from its recipe, the GPU
labels it (partition fingerprint = the oracle's, bit-exact) and solves the
spanning cluster's Kirchhoff system.  Each fixture holds the oracle's
solve at every decade 1e-8 ... 1e-17 or 1e-20 from ONE literal linbcg run
(round 3: or_linbcg_sym, bitwise the literal iterates), so it shows where
the reference solver has converged: the converged tolerance is the first
decade from which Gtop and Gbot move by < 2e-11 relative per decade
(CONV_STEP) to the end of the fixture.  Bars:

  * converged: Gtop and Gbot within 1e-10 relative of the oracle at that
    tolerance, for the default solve and the 4-slab row decomposition
    (SURVEY: "both within 1e-10 rel against the reference solver run at
    tol=1e-14 with itmax large" -- the fixtures show 1e-14 is not yet
    converged at the critical configs, so the bar is applied where the
    oracle itself has stopped moving).  The one widening, stated here and
    in DESIGN.md §5: where the reference solver ITSELF, re-run with only the
    association of its three dot products changed -- sums reversed (fixture
    "assoc_desc", make_config_golden.py --assoc) or pairwise / tree-summed
    like a GPU reduction ("assoc_tree", --assoc-tree) -- lands more than
    ASSOC_FLOOR away from the literal run, G is not defined to 1e-10 by the
    reference, and the bar is 1.5x the largest such spread (ASSOC_X).  This
    happens for Gtop at the critical bond configs (c2: 1024^2, c4: 2048^2,
    p = 0.5; Gtop is a sum of differences Va - V of top-row voltages within
    ~1e-6 of Va, resolved only to their fp64 spacing, gtop_resolution): the
    tree-summed oracle lands 1.66e-10 (c2) and 9.98e-10 (c4) away from the
    literal one, so the bars are 2.5e-10 and 1.5e-9.  That the GPU's own
    distance is association alone is shown separately: with the literal dot
    order (perc_set_dot_order, tests/test_literal_dot.py) the GPU solve is
    the literal oracle bitwise;
  * the reference tolerance 1e-8: iteration count within +-1 and G within
    twice the oracle's own truncation error there plus the tolerance (the
    solve is only accurate to |G(1e-8) - G(converged)|, and the dot
    products' association -- the only re-associated operations -- moves
    the iterates within that error), or 1.5x the re-associated oracles'
    spread at 1e-8 where that is larger (c4: the tree-summed run moves Gtop
    by 6.4e-8 at the same iteration count);
  * 1e-13: iteration count within +-3 (the recursive residual is near the
    fp64 floor) and the same truncation / association bar.
"""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

from percolation_amd import _lib as PL
from percolation_amd import api

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "configs", "*.json")))

CONVERGED = 1e-10

CONV_STEP = 2e-11  # per-decade change below which the oracle has converged
FLAT = 1e-10
ASSOC_FLOOR = 5e-11  # association spread of the reference solver above which it sets the bar


ASSOC_KEYS = ("assoc_desc", "assoc_tree")  # reversed serial sums; pairwise (tree) sums


ASSOC_X = 1.5  # bar = ASSOC_X x the reference solver's own association spread (where > ASSOC_FLOOR)


def gtop_resolution(doc, conv, Va=1.0, g0=1.0):
    """Relative change of Gtop when every top-row voltage moves by one ulp
    (an upper bound: all m bonds into the top electrode counted, 2m on the
    triangular lattice; only the spanning cluster's occupied ones carry
    current).

    Gtop sums g0 (Va - V_i) over the bonds into the top electrode
    (Square/bondc.f:554-592), with V_i within ~1e-6 of Va, so it can only
    resolve the V_i to their fp64 spacing just below Va (2^-53 for Va = 1).
    linbcg's x += ak p stalls on an element once the increments fall below
    half that spacing, so where the stall leaves each V_i depends on the
    iteration's rounding history -- the association of the dot products
    included -- while Gbot (voltages near 0, fine spacing) agrees to
    ~1e-12.  Explanatory only: the bars use the measured spreads."""
    rc = doc["recipe"]
    nb = rc["L"] * (2 if rc["lattice"] == 1 else 1)
    spacing = float(np.spacing(np.nextafter(Va, 0.0)))
    return nb * g0 * spacing / doc["solves"][conv]["gtop"]


def assoc_spread(doc, tkey, g):
    """the largest move of G at tolerance tkey over the re-associated oracle
    runs the fixture holds (0 if none ran to that tolerance)"""
    return max((rel(doc[k][tkey][g], doc["solves"][tkey][g]) for k in ASSOC_KEYS
                if tkey in doc.get(k, {})), default=0.0)


def iter_range(doc, tkey):
    """iteration counts of the literal oracle and its re-associated runs at
    tolerance tkey: (min, max)"""
    its = [doc["solves"][tkey]["iter"]] + [doc[k][tkey]["iter"] for k in ASSOC_KEYS
                                            if tkey in doc.get(k, {})]
    return min(its), max(its)


def iter_ok(doc, tkey, it):
    """the iteration count at a non-converged tolerance: +-1 while the
    recursive residual still tracks the true one (tol >= 1e-10); below that
    the stop decision rides on the rounding history (the fixtures' true
    residual has reached its floor at 1e-13: 0.8-2.8e-12), so the count must
    lie in the range the reference solver's own associations span (2 %
    slack, +-3); a fixture without re-associated runs takes the relative
    spread of the metric fixture (the same lattice class: L = 4096, bond p =
    0.6) at that tolerance -- its reversed sums stop 9.4 % later at 1e-13"""
    ref = doc["solves"][tkey]["iter"]
    if float(tkey) >= 1e-10:
        return abs(it - ref) <= 1
    if any(tkey in doc.get(k, {}) for k in ASSOC_KEYS):
        lo, hi = iter_range(doc, tkey)
        return 0.98 * lo - 3 <= it <= 1.02 * hi + 3
    metric = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs",
                                         "metric_sq4096_bond_p60.json")))
    lo, hi = iter_range(metric, tkey)
    spread = (hi - lo) / metric["solves"][tkey]["iter"]
    return abs(it - ref) <= max(3, 1.02 * spread * ref)


def converged_bar(doc, conv, g):
    """FLAT; or ASSOC_X x the reference solver's own association spread at
    the converged tolerance where that exceeds ASSOC_FLOOR (module
    docstring)"""
    spread = assoc_spread(doc, conv, g)
    return max(FLAT, ASSOC_X * spread) if spread > ASSOC_FLOOR else FLAT


def test_association_spread_is_gtop_resolution_noise():
    """CPU: at the deepest decade of every fixture (where the runs have
    stopped moving) the reference solver's re-associated runs move Gtop by at
    most 4 units of its top-row resolution (c4's tree sums: 3.2) and Gbot by
    < 1e-12 -- the spread the bars are built from is the fp64 resolution of
    Gtop, not a difference in the per-row arithmetic"""
    for f in FIXTURES:
        doc = json.load(open(f))
        deep = min(doc["solves"], key=float)
        res = gtop_resolution(doc, deep)
        for k in ASSOC_KEYS:
            if deep in doc.get(k, {}):
                assert rel(doc[k][deep]["gtop"], doc["solves"][deep]["gtop"]) < 4 * res, (f, k)
                assert rel(doc[k][deep]["gbot"], doc["solves"][deep]["gbot"]) < 1e-12, (f, k)


def test_iteration_ranges_at_the_converged_decade():
    """CPU: the BASELINE config fixtures hold re-associated runs at their
    converged decade, so the GPU's iteration count there is checked against a
    range the reference solver itself spans (the bench realisation's fixture,
    one L = 4096 solve of hours, holds the literal run only)"""
    for f in FIXTURES:
        doc = json.load(open(f))
        conv = converged_tol(doc["solves"])
        if not os.path.basename(f).startswith("bench_"):
            assert any(conv in doc.get(k, {}) for k in ASSOC_KEYS), f
        lo, hi = iter_range(doc, conv)
        assert lo <= doc["solves"][conv]["iter"] <= hi


def test_bars_are_the_reference_spread():
    """CPU: the converged bars are flat 1e-10 except where the reference's
    own association spread sets them, and never wider than 1.5e-9"""
    for f in FIXTURES:
        doc = json.load(open(f))
        conv = converged_tol(doc["solves"])
        for g in ("gtop", "gbot"):
            bar = converged_bar(doc, conv, g)
            sp = assoc_spread(doc, conv, g)
            assert bar == FLAT or bar == ASSOC_X * sp, (f, g, bar, sp)
            assert bar < 1.6e-9, (f, g, bar)


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def converged_tol(solves):
    """the first tolerance from which every further decade moves Gtop and
    Gbot by < CONV_STEP (None if the fixture never gets there)"""
    tols = sorted(solves, key=float, reverse=True)  # loose -> tight
    steps = [max(rel(solves[b]["gtop"], solves[a]["gtop"]), rel(solves[b]["gbot"], solves[a]["gbot"]))
             for a, b in zip(tols, tols[1:])]
    for i in range(len(steps)):
        if all(x < CONV_STEP for x in steps[i:]):
            return tols[i + 1]
    return None


def occupation(rc):
    lat, L_, p = rc["lattice"], rc["L"], rc["p"]
    if rc["kind"] == "bond":
        seed = rc["tseed"]
        nb = api.nbonds(lat, L_, L_, 0)
        tb = int(p * nb)
        if rc["order"] == "ref":
            ids = api.shuffled_ids(nb, seed)
        elif rc["order"] == "device":  # drawn on the GPU, as bench.py times it
            return dict(device=(PL.BOND, 0, tb, seed)), PL.RULE_BOND, PL.CUR_FORTRAN
        else:
            ids = (np.random.default_rng(seed).permutation(nb)[:tb] + 1).astype(np.int32)
        return dict(kind=PL.BOND, bond_order=ids, nbonds_=tb), PL.RULE_BOND, PL.CUR_FORTRAN
    t = L_ * L_
    if rc["kind"] == "mixed":  # sitebond.f: sites (sseed) then bonds (bseed), reference shuffles
        nb = api.nbonds(lat, L_, L_, 0)
        return (dict(kind=PL.SITEBOND, site_order=api.shuffled_ids(t, rc["sseed"]),
                     nsites=int(p * t), bond_order=api.shuffled_ids(nb, rc["bseed"]),
                     nbonds_=int(rc["pb"] * nb)), PL.RULE_MIXED, PL.CUR_MATLAB)
    ts = int(p * t)
    return (dict(kind=PL.SITE, site_order=api.shuffled_ids(t, rc["tseed"]), nsites=ts),
            PL.RULE_SITE, PL.CUR_MATLAB)


def test_converged_tol_rule():
    """CPU: the converged-decade rule on synthetic histories, and every
    committed fixture reaches convergence"""
    mk = lambda *g: {"1e-%d" % (8 + i): dict(gtop=1.0 + a, gbot=1.0 + b) for i, (a, b) in enumerate(g)}
    assert converged_tol(mk((0, 0), (1e-9, 0), (1e-9 + 1e-12, 5e-12), (1e-9 + 1e-12, 5e-12))) == "1e-10"
    assert converged_tol(mk((0, 0), (1e-9, 0), (2e-9, 0))) is None
    assert converged_tol(mk((0, 0), (0, 0))) == "1e-9"
    for f in FIXTURES:
        assert converged_tol(json.load(open(f))["solves"]) is not None, f


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(f)[:-5] for f in FIXTURES])
def test_config_fixture(path):
    doc = json.load(open(path))
    rc = doc["recipe"]
    occ, rule, cur = occupation(rc)
    L_ = rc["L"]
    solves = doc["solves"]
    conv = converged_tol(solves)
    assert conv is not None, "fixture not converged: regenerate it deeper (make_config_golden.py)"
    runs = [t for t in ("1e-08", "1e-13") if t in solves] + [conv]
    report = {}
    with api.Context(rc["lattice"], L_, L_, 0) as ctx:
        if "device" in occ:
            ctx.occupy_random(*occ["device"])
        else:
            ctx.occupy(**occ)
        li = ctx.label(canon=True)
        h = hashlib.sha256(np.ascontiguousarray(li["canon"], dtype=np.int32).tobytes()).hexdigest()
        assert h == doc["label"]["canon_sha256"], "partition differs from the oracle's"
        assert li["nspan"] > 0
        for tkey in runs:
            ref = solves[tkey]
            c = ctx.conductance(rule, cur, tol=float(tkey), itmax=10 ** 6)
            report[tkey] = d = dict(tol=tkey, iter=c["iter"], iter_ref=ref["iter"],
                                    gtop_rel=rel(c["gtop"], ref["gtop"]),
                                    gbot_rel=rel(c["gbot"], ref["gbot"]))
            print(json.dumps(d))
        # the row-slab solve (perc_set_slabs, 4 slabs) against the converged fixture
        ctx.set_slabs(4)
        c = ctx.conductance(rule, cur, tol=float(conv), itmax=10 ** 6)
        ctx.set_slabs(1)
        ref = solves[conv]
        report["slabs"] = d = dict(tol=conv + " (4 slabs)", iter=c["iter"], iter_ref=ref["iter"],
                                   gtop_rel=rel(c["gtop"], ref["gtop"]),
                                   gbot_rel=rel(c["gbot"], ref["gbot"]))
        print(json.dumps(d))
    for key in (conv, "slabs"):  # converged: 1e-10 on both conductances (see converged_bar)
        d = report[key]
        for g in ("gtop", "gbot"):
            assert d[g + "_rel"] < converged_bar(doc, conv, g), (g, converged_bar(doc, conv, g), d)
        # past ~1e-15 the stop decision rides on the rounding history: the
        # iteration count must lie in the range the reference solver's own
        # associations span at that decade (literal, reversed, tree sums), 2 % slack
        if any(conv in doc.get(k, {}) for k in ASSOC_KEYS):
            lo, hi = iter_range(doc, conv)
            assert 0.98 * lo <= d["iter"] <= 1.02 * hi, (d, lo, hi)
    for tkey in runs:
        if tkey == conv:
            continue
        d, ref, cv = report[tkey], solves[tkey], solves[conv]
        assert iter_ok(doc, tkey, d["iter"]), d
        for g in ("gtop", "gbot"):
            # the oracle's own error at this tol, plus the tolerance itself:
            # where G has converged ahead of the residual (the metric's Gtop
            # moves 3.6e-10 from 1e-8 to 1e-13), stopping one iteration
            # apart still moves it by the last step (1.4e-9 there)
            # (or the re-associated oracles' own spread at this tol, if larger)
            trunc = rel(ref[g], cv[g])
            bar = max(2 * trunc + max(1e-10, float(tkey)), ASSOC_X * assoc_spread(doc, tkey, g))
            assert d[g + "_rel"] <= bar, (g, trunc, bar, d)


@pytest.mark.gpu
def test_literal_c5m_fixture_bitwise():
    """Config 5's rule at a size the oracle solves (c5m: 1024^2 square mixed
    site-then-bond, ps = pb = 0.85, ConductCalc.m:134-160) in the literal dot
    order through the PRODUCTION march (q-free, strip-major, nibble codes,
    tagged reductions; PERC_DOT_LITERAL_HOST: the serial sums of the
    kernels' own terms formed by the host, bitwise the GPU fold): iter, err,
    Gtop, Gbot and every committed err-history point are the oracle
    fixture's bitwise at the reference tolerance 1e-8 (5 193 iterations;
    Square/bondc.f:750-838).  The GPU record of the same run at the other
    config sizes: profiles/r5_4_literal_*, r6_1_literal_metric_*."""
    doc = json.load(open(os.path.join(HERE, "golden", "configs", "c5m_sq1024_mixed_p85.json")))
    rc = doc["recipe"]
    occ, rule, cur = occupation(rc)
    ref = doc["solves"]["1e-08"]
    with api.Context(rc["lattice"], rc["L"], rc["L"], 0) as ctx:
        ctx.set_march_mode(PL.MARCH_DEFAULT & ~PL.SOLVE_RESIDENT)
        ctx.occupy(**occ)
        assert ctx.label()["nspan"] > 0
        ctx.set_dot_order(PL.DOT_LITERAL_HOST)
        c = ctx.conductance(rule, cur, tol=1e-8, itmax=10 ** 6)
        hist = ctx.err_history()
        ran = ctx.last_solve()
    assert ran["kernel"] == "march" and ran["lit_terms"] and ran["host_fold"], ran
    assert ran["qfree"] and ran["strips"] and ran["nibble"] and ran["tag"], ran
    assert (c["iter"], c["err"], c["gtop"], c["gbot"]) == (ref["iter"], ref["err"], ref["gtop"], ref["gbot"]), \
        (c, ref["iter"], ref["gtop"], ref["gbot"])
    assert all(hist[k - 1] == e for k, e in ref["err_history"])
