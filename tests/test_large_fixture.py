"""Config 5's near-critical companion at its own size, against the oracle:
8192^2 square mixed site-then-bond at ps = pb = 0.85 (ConductCalc.m:134-160
mixed rule), both occupations drawn on the GPU by perc_occupy_random
(PERC_SITEBOND, seed 777), as tools/l8192_probe.py and bench.py's companion
line run it.  Its vectors are past the 256 MB Infinity Cache, so the
production solver is the ROW-MAJOR q-free march (P and B on nibble codes):
the solver no other fixture reaches at its production size.

The fixture (tests/golden/large/c5c_sq8192_mixed_p85_dev.json, made by
tests/golden/make_config_golden.py --decades with GOLDEN_PREFIX from the
oracle's literal linbcg, Square/bondc.f:750-838, on this container's CPU)
holds the partition fingerprint and the complete err history of the first
iterations.  With the literal dot order the GPU's production kernels store
their rows' dot terms and the host folds them in ascending j
(PERC_DOT_LITERAL_HOST), so every err of the prefix must be the oracle's
bitwise; the full 67 M-row literal solve (~2 min per 1000 iterations) is
run once as a profile, profiles/r6_*_literal_c5c_*.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from percolation_amd import _lib as PL
from percolation_amd import api

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "large", "c5c_sq8192_mixed_p85_dev.json")
PREFIX_GPU = 200  # iterations the -m gpu test runs (~125 ms each in the literal order at 67 M rows)


def fixture():
    if not os.path.exists(FIX):
        pytest.skip("no large fixture")
    return json.load(open(FIX))


def test_large_fixture_recipe():
    """CPU: the fixture is the companion's recipe and holds a prefix"""
    doc = fixture()
    rc = doc["recipe"]
    assert (rc["lattice"], rc["L"], rc["kind"], rc["p"], rc["pb"], rc["order"], rc["seed"]) == \
        (0, 8192, "mixed", 0.85, 0.85, "device", 777)
    assert len(doc["err_prefix"]) >= PREFIX_GPU
    assert doc["label"]["perccln"] > 0


@pytest.mark.gpu
def test_rowmajor_march_prefix_is_the_oracle_bitwise():
    doc = fixture()
    rc = doc["recipe"]
    L_ = rc["L"]
    t = L_ * L_
    nb = api.nbonds(0, L_, L_, 0)
    ts, tb = int(rc["p"] * t), int(rc["pb"] * nb)
    pre = np.array(doc["err_prefix"][:PREFIX_GPU], dtype=np.float64)
    with api.Context(0, L_, L_, 0) as ctx:
        ctx.occupy_random(PL.SITEBOND, ts, tb, rc["seed"])
        li = ctx.label(canon=True)
        h = hashlib.sha256(np.ascontiguousarray(li["canon"], dtype=np.int32).tobytes()).hexdigest()
        assert h == doc["label"]["canon_sha256"], "partition differs from the oracle's"
        assert li["nspan"] > 0
        ctx.set_march_mode(PL.MARCH_DEFAULT & ~PL.SOLVE_RESIDENT)
        ctx.set_dot_order(PL.DOT_LITERAL_HOST)
        c = ctx.conductance(PL.RULE_MIXED, PL.CUR_MATLAB, tol=1e-300, itmax=len(pre) - 1)
        hist = ctx.err_history()
        ran = ctx.last_solve()
    # the L > 4096 production kernels: q-free, row-major, nibble codes, their own terms
    assert ran["kernel"] == "march" and ran["qfree"] and not ran["strips"] and ran["nibble"], ran
    assert ran["lit_terms"] and ran["host_fold"], ran
    assert c["iter"] == len(pre)
    assert np.array_equal(np.asarray(hist[:len(pre)]).view(np.uint64), pre.view(np.uint64))


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


@pytest.mark.gpu
def test_rowmajor_default_solve_within_the_oracle_bars():
    """The default (fast dot order) solve of the companion -- the row-major
    q-free march with its ticket reductions, as bench.py's companion
    line runs it -- against the oracle's literal linbcg at the reference
    tolerance 1e-8: the iteration count within +-1 (the recursive residual
    still tracks the true one there) and Gtop / Gbot within twice the
    oracle's own move from 1e-8 to 1e-9 plus the tolerance (the bar of
    tests/test_config_goldens.py at 1e-8, with the 1e-9 decade standing in
    for the converged one this 67 M-row fixture does not reach: hours of
    CPU per decade)."""
    doc = fixture()
    if "1e-08" not in doc["solves"] or "1e-09" not in doc["solves"]:
        pytest.skip("fixture without the 1e-8 / 1e-9 decades")
    rc = doc["recipe"]
    L_ = rc["L"]
    t = L_ * L_
    nb = api.nbonds(0, L_, L_, 0)
    ref, nxt = doc["solves"]["1e-08"], doc["solves"]["1e-09"]
    with api.Context(0, L_, L_, 0) as ctx:
        ctx.occupy_random(PL.SITEBOND, int(rc["p"] * t), int(rc["pb"] * nb), rc["seed"])
        assert ctx.label()["nspan"] > 0
        c = ctx.conductance(PL.RULE_MIXED, PL.CUR_MATLAB, tol=1e-8, itmax=10 ** 6)
        ran = ctx.last_solve()
    assert ran["kernel"] == "march" and ran["qfree"] and not ran["strips"] and ran["nibble"], ran
    assert not ran["literal"], ran
    assert abs(c["iter"] - ref["iter"]) <= 1, (c["iter"], ref["iter"])
    for g in ("gtop", "gbot"):
        bar = 2 * rel(ref[g], nxt[g]) + 1e-8
        assert rel(c[g], ref[g]) <= bar, (g, c[g], ref[g], bar)
