"""Pin the CPU oracle (oracle/perc_oracle.c) to the reference.

Fixtures under tests/golden/ were produced by the compiled reference Fortran
(oracle/build_ref.sh + tests/golden/make_golden.py).  Everything here is
bit-exact: byte-identical output files, bitwise-equal Gtop/Gbot/Vint and
per-iteration linbcg err.
"""
import ctypes as C
import os

import numpy as np
import pytest

import golden_io as G
from percolation_amd import api
import oracle_lib as O

BONDC = [v for v in G.variants() if G.meta(v)["kind"] == "bondc"]
SITE = [v for v in G.variants() if G.meta(v)["kind"] == "site"]
SITEBOND = [v for v in G.variants() if G.meta(v)["kind"] == "sitebond"]
BONDCOND = [v for v in G.variants() if G.meta(v)["kind"] == "bond_cond"]
BONDSITE = [v for v in G.variants() if G.meta(v)["kind"] == "bondsite"]

LIBGFORTRAN = "/opt/conda/lib/libgfortran.so.4"


@pytest.mark.skipif(not os.path.exists(LIBGFORTRAN), reason="libgfortran absent")
def test_rng_matches_libgfortran():
    """or_rand/or_srand == GNU Fortran runtime rand/srand (L0 in SURVEY.md)."""
    gf = C.CDLL(LIBGFORTRAN)
    gf._gfortran_rand.restype = C.c_float
    gf._gfortran_rand.argtypes = [C.POINTER(C.c_int)]
    gf._gfortran_srand.argtypes = [C.POINTER(C.c_int)]
    L = O.lib()
    zero = C.c_int(0)
    for seed in (626504, 62703, 1080115, 58302, 1, 0, 2147483646, 4562929):
        s = C.c_int(seed)
        gf._gfortran_srand(C.byref(s))
        L.or_srand(seed)
        a = np.array([gf._gfortran_rand(C.byref(zero)) for _ in range(20000)], np.float32)
        b = np.array([L.or_rand(0) for _ in range(20000)], np.float32)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), seed
    # rand(1) restarts the sequence, rand(k>1) reseeds (randtest.f:32-39)
    for arg in (1, 7, 12345):
        a = gf._gfortran_rand(C.byref(C.c_int(arg)))
        b = L.or_rand(arg)
        assert np.float32(a) == np.float32(b)


def test_trial_seeds():
    """tseed(1) from master 58302 (Square/bond_cond.f:65-70)."""
    ts = O.i32(1000)
    O.lib().or_trial_seeds(58302, 1000, ts)
    assert ts[0] == 4562929
    for v in BONDCOND:
        txt = G.text(v, "bondcond.txt").decode()
        seeds = [int(l.split(":")[1]) for l in txt.splitlines() if "Random number seed" in l]
        assert list(ts[:len(seeds)]) == seeds


@pytest.mark.parametrize("lattice,m,n,pbc", [(0, 50, 50, 0), (0, 50, 50, 1), (1, 50, 50, 0),
                                             (1, 50, 50, 1), (0, 64, 64, 0), (1, 10, 10, 0)])
def test_bond_list_count(lattice, m, n, pbc):
    L = O.lib()
    b1, b2 = O.bond_list(lattice, m, n, pbc)
    assert np.all(b1 < b2)
    assert np.all(np.diff(b1) >= 0)
    nb = L.or_nbonds(lattice, m, n, pbc)
    assert len(b1) == nb


@pytest.mark.parametrize("v", [v for v in SITE])
def test_bondlist_file(v):
    p = G.meta(v)["params"]
    b1, b2 = O.bond_list(p["lattice"], p["m"], p["n"], p["pbc"])
    assert G.fmt_i10(b1, b2) == G.text(v, "bondlist.txt")


@pytest.mark.parametrize("v", BONDC)
def test_bondorder_file(v):
    p = G.meta(v)["params"]
    b1, b2, o1, o2 = O.bond_order(p["lattice"], p["m"], p["n"], p["pbc"], p["seed"])
    nb = len(b1)
    assert G.fmt_i10(o1[:nb], o2[:nb]) == G.text(v, "bondorder.txt")


@pytest.mark.parametrize("literal", [True, False])
@pytest.mark.parametrize("v", BONDC)
def test_bond_labels(v, literal):
    """bond.txt byte-identical: b1,b2,label,j,c(j) (Square/bondc.f:600-604)."""
    md = G.meta(v)
    p = md["params"]
    b1, b2, o1, o2 = O.bond_order(p["lattice"], p["m"], p["n"], p["pbc"], p["seed"])
    nb = len(b1)
    tb = int(p["pb"] * nb)
    label, csize, cln, mx, ms = O.label_bonds(p["lattice"], p["m"], p["n"], p["pbc"],
                                              b1, b2, o1, o2, tb, literal=literal)
    assert cln > 0
    got = G.fmt_i10(b1, b2, label, np.arange(1, nb + 1), csize[1:nb + 1])
    assert got == G.text(v, "bond.txt")
    assert (mx, ms) == (md["maxcn"], md["maxcs"])
    L = O.lib()
    span = L.or_span_bonds(p["m"], p["n"], nb, b1, b2, label, csize, cln)
    assert span == md["perccln"]
    if span:
        assert csize[span] == md["perccls"]


@pytest.mark.parametrize("v", BONDC)
def test_bondc_conductance_bitwise(v):
    """assembly + linbcg + currents bitwise (Square/bondc.f:465-595)."""
    md = G.meta(v)
    p = md["params"]
    if not md["perccln"]:
        pytest.skip("no spanning cluster")
    r = O.bondc(p["lattice"], p["m"], p["n"], p["pbc"], p["pb"], p["seed"],
                tol=p.get("tol", 1e-8), itmax=p.get("itmax", 2500))
    assert r["perccln"] == md["perccln"]
    assert r["iter"] == md["iter"]
    assert r["gtop"] == md["gtop"] and r["gbot"] == md["gbot"], (r["gtop"], r["gbot"])
    # per-iteration err and Vint where printed
    b1, b2, o1, o2 = O.bond_order(p["lattice"], p["m"], p["n"], p["pbc"], p["seed"])
    gval = O.f64(len(b1))
    O.lib().or_bond_values(0, len(b1), b1, b2, r["label"], O.i32(1), r["perccln"], 1.0,
                           1e-12, gval)
    c = O.conductance(p["lattice"], p["m"], p["n"], p["pbc"], b1, b2, gval,
                      tol=p.get("tol", 1e-8), itmax=p.get("itmax", 2500))
    assert np.array_equal(c["errs"], np.array(md["linbcg_err"]))
    if "vint" in md:
        assert np.array_equal(c["vint"], np.array(md["vint"]))


@pytest.mark.parametrize("literal", [True, False])
@pytest.mark.parametrize("v", SITE)
def test_site_labels(v, literal):
    """site.txt / siteorder.txt byte-identical (Square/site.f:131-359)."""
    md = G.meta(v)
    p = md["params"]
    t = p["m"] * p["n"]
    order = O.site_order(t, p["seed"])
    got_order = "".join(" %d\n" % x for x in order[:t]).encode()
    assert got_order == G.text(v, "siteorder.txt")
    ts = int(p["ps"] * t)
    s, csize, cln, mx, ms = O.label_sites(p["lattice"], p["m"], p["n"], p["pbc"], order, ts,
                                          literal=literal)
    got = G.fmt_i10(np.arange(1, t + 1), s, csize[1:t + 1])
    assert got == G.text(v, "site.txt")
    assert (mx, ms) == (md["maxcn"], md["maxcs"])
    span = O.lib().or_span_sites(p["m"], p["n"], s, csize, cln, p["n"])
    assert span == md["perccln"]


@pytest.mark.parametrize("v", SITEBOND)
def test_sitebond_labels(v):
    """sbsite.txt / sbbond.txt byte-identical (Square/sitebond.f:187-477)."""
    md = G.meta(v)
    p = md["params"]
    lat, m, n, pbc = p["lattice"], p["m"], p["n"], p["pbc"]
    t = m * n
    L = O.lib()
    sorder = O.site_order(t, p["sseed"])
    b1, b2, o1, o2 = O.bond_order(lat, m, n, pbc, p["bseed"])
    nb = len(b1)
    ts, tb = int(p["ps"] * t), int(p["pb"] * nb)
    s, bl, cs = O.i32(t), O.i32(nb), O.i32(t + nb + 2)
    mx, ms = C.c_int(), C.c_int()
    cln = L.or_label_sitebond(lat, m, n, pbc, nb, b1, b2, sorder, ts, o1, o2, tb, s, bl, cs,
                              C.byref(mx), C.byref(ms))
    assert G.fmt_i10(np.arange(1, t + 1), s, cs[1:t + 1]) == G.text(v, "sbsite.txt")
    assert G.fmt_i10(b1, b2, bl) == G.text(v, "sbbond.txt")
    assert (mx.value, ms.value) == (md["maxcn"], md["maxcs"])
    assert L.or_span_sites(m, n, s, cs, cln, 2 * n - 1) == md["perccln"]


@pytest.mark.parametrize("v", BONDSITE)
def test_bondsite_labels(v):
    """bssite.txt / bsbond.txt byte-identical (Square/bondsite.f:170-430),
    the oracle's literal loops and libperc's O(N alpha) replay alike."""
    md = G.meta(v)
    p = md["params"]
    lat, m, n, pbc = p["lattice"], p["m"], p["n"], p["pbc"]
    t = m * n
    L = O.lib()
    b1, b2 = O.bond_list(lat, m, n, pbc)
    nb = len(b1)
    sorder = O.site_order(t, p["sseed"])
    border = O.site_order(nb, p["bseed"])  # shuffled bond ids (0: spill slot)
    ts, tb = int(p["ps"] * t), int(p["pb"] * nb)
    s, bl, cs = O.i32(t), O.i32(nb), O.i32(t + nb + 2)
    mx, ms = C.c_int(), C.c_int()
    cln = L.or_label_bondsite(lat, m, n, pbc, nb, b1, b2, border, tb, sorder, ts, s, bl, cs,
                              C.byref(mx), C.byref(ms))
    s_ext = np.zeros(nb, dtype=np.int64)
    s_ext[:min(t, nb)] = s[:min(t, nb)]
    assert G.fmt_i10(np.arange(1, nb + 1), s_ext, cs[1:nb + 1]) == G.text(v, "bssite.txt")
    assert G.fmt_i10(b1, b2, bl) == G.text(v, "bsbond.txt")
    assert (mx.value, ms.value) == (md["maxcn"], md["maxcs"])
    assert L.or_span_sites(m, n, s, cs, cln, 2 * n - 1) == md["perccln"]
    r = api.bondsite(lat, m, n, pbc, p["ps"], p["pb"], p["sseed"], p["bseed"])
    assert r["bssite"].encode() == G.text(v, "bssite.txt")
    assert r["bsbond"].encode() == G.text(v, "bsbond.txt")
    assert (r["maxcn"], r["maxcs"], r["perccln"]) == (md["maxcn"], md["maxcs"], md["perccln"])


@pytest.mark.parametrize("v", BONDCOND)
def test_bond_cond_rows(v):
    """bond_cond sweep rows (f12.9) and pc (Square/bond_cond.f:123-505)."""
    md = G.meta(v)
    p = md["params"]
    txt = G.text(v, "bondcond.txt").decode().splitlines()
    ts = O.i32(1000)
    L = O.lib()
    L.or_trial_seeds(p["seed"], 1000, ts)
    trials, cur = [], None
    for line in txt:
        if "Trial #" in line:
            cur = {"rows": []}
            trials.append(cur)
        elif cur is not None and line.count(",") == 3:
            cur["rows"].append(line)
        elif "lattice-spanning cluster:" in line:
            cur["perccln"] = int(line.split(":")[1])
        elif "pc =" in line:
            cur["pc"] = float(line.split("=")[1])
    assert len(trials) == p["numtrials"]
    for ii, tr in enumerate(trials):
        pb, gb, gt = O.f64(250), O.f64(250), O.f64(250)
        it = O.i32(250)
        pc = C.c_double()
        perc = C.c_int()
        nrow = L.or_bond_cond_trial(p["lattice"], p["m"], p["n"], p["pbc"], int(ts[ii]), 1.0,
                                    1.0, 2500, 1e-8, pb, gb, gt, it, C.byref(perc),
                                    C.byref(pc))
        rows = [" %11.9f,%12.9f,%12.9f,%12.9f" % (pb[k], gb[k], gt[k], (gb[k] + gt[k]) / 2)
                for k in range(nrow)]
        assert rows == tr["rows"]
        assert perc.value == tr["perccln"]
        assert pc.value == tr["pc"]
