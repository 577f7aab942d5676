"""The Fortran drivers (percolation_amd/fortran, drop-ins for the reference
programs) against the reference's own output files (tests/golden, made by
the flang-compiled reference).

* bondorder.txt, bond.txt, siteorder.txt, bondlist.txt, site.txt,
  sbsite.txt, sbbond.txt: byte-identical.
* bondcond.txt: every text line identical (header, trial seeds, pb column,
  spanning label, pc); the conductance columns (f12.9) agree to the printed
  precision (the GPU PCG and the reference agree to ~1e-10 rel, and at
  tol 1e-8 the reference's own Gbot is off the converged value by up to
  ~3e-7 -- compared at 2e-9 like tests/test_gpu_parity.py).
* bondc's printed conductance: Gtop within 1e-10 rel of the reference.
* Without a device the drivers stop with PERC_ENODEV -- no CPU fallback --
  after writing the host-side outputs (bondorder.txt).
"""
import os
import shutil
import subprocess

import pytest

import golden_io as G
from percolation_amd import _lib as PL
from percolation_amd import api

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "percolation_amd", "fortran", "bin")
TRACES = {"bondocc.txt", "siteocc.txt", "sbdebug.txt", "bsdebug.txt"}  # per-step logs (trace = 1 only)
# golden kind -> (program, namelist group, parameters)
NML = {"bondc": ("bondc", "bondc", ("lattice", "m", "n", "pbc", "pb", "seed", "tol", "itmax")),
       "site": ("site", "site", ("lattice", "m", "n", "pbc", "ps", "seed")),
       "sitebond": ("sitebond", "sitebond",
                    ("lattice", "m", "n", "pbc", "ps", "pb", "sseed", "bseed")),
       "bondsite": ("bondsite", "bondsite",
                    ("lattice", "m", "n", "pbc", "ps", "pb", "sseed", "bseed")),
       "bond_cond": ("bond_cond", "bond_cond", ("lattice", "m", "n", "pbc", "numtrials", "seed")),
       "bond_perc": ("bond_perc", "perc_scan", ("lattice", "m", "n", "pbc", "numtrials", "seed")),
       "site_perc": ("site_perc", "perc_scan", ("lattice", "m", "n", "pbc", "numtrials", "seed")),
       "sb_perc": ("sb_perc", "mixed_scan", ("lattice", "m", "n", "pbc", "seed", "iters")),
       "bs_perc": ("bs_perc", "mixed_scan", ("lattice", "m", "n", "pbc", "seed", "iters"))}


def exe(prog, lattice):
    path = os.path.join(BIN, "%s_%s" % (prog, "tri" if lattice else "sq"))
    if not os.path.exists(path):
        pytest.skip("Fortran drivers not built (percolation_amd/fortran: make)")
    return path


def run_variant(v, tmp_path, expect_ok=True, extra=()):
    md = G.meta(v)
    prog, group, keys = NML[md["kind"]]
    p = md["params"]
    items = []
    for k in keys:
        if k in p:
            val = p[k]
            items.append("%s=%s" % (k, repr(float(val)) if isinstance(val, float) else int(val)))
    if "points" in p:  # psarray(i) = pstart + pstep*(i-1), as edited in oracle/build_ref.sh
        pts = p["points"]
        items += ["pstart=%r" % round(pts[0], 6), "pstep=%r" % round(pts[1] - pts[0], 6),
                  "npoints=%d" % len(pts)]
    items += list(extra)
    (tmp_path / ("%s.nml" % prog)).write_text("&%s_nml %s /\n" % (group, ", ".join(items)))
    r = subprocess.run([exe(prog, p["lattice"])], cwd=tmp_path, capture_output=True, text=True,
                       timeout=600)
    if expect_ok:
        assert r.returncode == 0, r.stderr[-2000:]
    return md, r


def golden_files(v):
    d = os.path.join(G.GOLDEN, v)
    return sorted(f[:-3] for f in os.listdir(d) if f.endswith(".gz") and f[:-3] not in TRACES)


def have_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def test_driver_without_device_fails_loudly(tmp_path):
    """No HIP device: bondorder.txt (host RNG + shuffle) is written and equals
    the reference's, then the driver stops with PERC_ENODEV (-8)."""
    if have_gpu():
        pytest.skip("a device is present")
    if shutil.which(os.path.join(BIN, "bondc_sq")) is None:
        pytest.skip("Fortran drivers not built")
    md, r = run_variant("sq_bondc_p60", tmp_path, expect_ok=False)
    assert r.returncode != 0
    assert "status -8" in r.stderr
    assert (tmp_path / "bondorder.txt").read_bytes() == G.text("sq_bondc_p60", "bondorder.txt")
    assert not (tmp_path / "bond.txt").exists()


FILE_VARIANTS = [v for v in G.variants()
                 if G.meta(v)["kind"] in ("bondc", "site", "sitebond", "bond_perc", "site_perc",
                                          "sb_perc", "bs_perc")]


@pytest.mark.gpu
@pytest.mark.parametrize("v", FILE_VARIANTS)
def test_driver_outputs_byte_identical(v, tmp_path):
    md, r = run_variant(v, tmp_path)
    files = golden_files(v)
    assert files
    for f in files:
        assert (tmp_path / f).read_bytes() == G.text(v, f), f
    if md["kind"] == "bondc" and md.get("perccln"):
        line = [l for l in r.stdout.splitlines() if "Conductance:" in l][-1]
        gtop, gbot = (float(x) for x in line.split(":")[1].split())
        assert abs(gtop - md["gtop"]) <= 1e-10 * abs(md["gtop"])
        tight = md["params"].get("tol", 1e-8) <= 1e-13
        assert abs(gbot - md["gbot"]) <= (1e-10 if tight else 1e-6) * abs(md["gbot"])


@pytest.mark.parametrize("v", [v for v in G.variants() if G.meta(v)["kind"] == "bondsite"])
def test_bondsite_driver_byte_identical(v, tmp_path):
    """bondsite (host replay through the Fortran binding; the reference
    computes no conductance there, so no device): bssite.txt and bsbond.txt
    byte-identical, largest / spanning cluster as printed."""
    md, r = run_variant(v, tmp_path)
    for f in golden_files(v):
        assert (tmp_path / f).read_bytes() == G.text(v, f), f
    assert "largest overall cluster size: %d" % md["maxcs"] in " ".join(r.stdout.split())
    if md["perccln"]:
        assert "infinite cluster number: %d" % md["perccln"] in " ".join(r.stdout.split())


@pytest.mark.gpu
@pytest.mark.parametrize("v", [v for v in G.variants() if G.meta(v)["kind"] == "bond_cond"])
def test_bond_cond_driver(v, tmp_path):
    run_variant(v, tmp_path)
    got = (tmp_path / "bondcond.txt").read_text().splitlines()
    want = G.text(v, "bondcond.txt").decode().splitlines()
    assert len(got) == len(want)
    for a, b in zip(got, want):
        if b.count(",") == 3:  # pb, Gbot, Gtop, mean  (f12.9)
            fa, fb = [float(x) for x in a.split(",")], [float(x) for x in b.split(",")]
            assert a.split(",")[0] == b.split(",")[0]
            assert all(abs(x - y) <= 2e-9 for x, y in zip(fa[1:], fb[1:])), (a, b)
        else:
            assert a == b


@pytest.mark.gpu
@pytest.mark.parametrize("v", ["sq_bondc_p60", "tri_bondc_p35", "sq_bondc_p60_tight"])
def test_bondc_driver_literal_dot_order(v, tmp_path):
    """dot_order = 1 (perc_set_dot_order): the driver's printed conductance
    and iteration count are the reference solver's exactly"""
    md, r = run_variant(v, tmp_path, extra=["dot_order=1"])
    for f in golden_files(v):
        assert (tmp_path / f).read_bytes() == G.text(v, f), f
    line = [l for l in r.stdout.splitlines() if "Conductance:" in l][-1]
    gtop, gbot = (float(x) for x in line.split(":")[1].split())
    assert gtop == md["gtop"] and gbot == md["gbot"], (gtop, gbot, md["gtop"], md["gbot"])
    it = [l for l in r.stdout.splitlines() if "linbcg iterations:" in l][-1]
    assert int(it.split(":")[1].split()[0]) == md["iter"]


@pytest.mark.gpu
@pytest.mark.parametrize("nslab", [2, 3])
def test_bondc_driver_split_solve(nslab, tmp_path):
    """nslab > 1 (perc_dslab_solve_group from the Fortran host; xport 1: the
    contexts share the box's one GPU; the slab kernels need m a multiple of
    128): bond.txt byte-identical to the one-context run and the
    conductance the one-context solve's to 1e-10 at tol 1e-13"""
    prog = exe("bondc", 0)
    out = {}
    for k in (1, nslab):
        d = tmp_path / ("k%d" % k)
        d.mkdir()
        (d / "bondc.nml").write_text("&bondc_nml lattice=0, m=256, n=200, pbc=0, pb=0.6, "
                                     "seed=626504, tol=1e-13, itmax=100000, nslab=%d, xport=1 /\n" % k)
        r = subprocess.run([prog], cwd=d, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [l for l in r.stdout.splitlines() if "Conductance:" in l][-1]
        out[k] = [float(x) for x in line.split(":")[1].split()] + [(d / "bond.txt").read_bytes()]
    (g1, b1, t1), (gk, bk, tk) = out[1], out[nslab]
    assert t1 == tk
    assert abs(gk - g1) <= 1e-10 * abs(g1) and abs(bk - b1) <= 1e-10 * abs(b1), (out[1][:2], out[nslab][:2])


@pytest.mark.gpu
@pytest.mark.parametrize("extra", ["", "dot_order=1", "condtype=2"])
def test_bondc_driver_split_solve_falls_back(extra, tmp_path):
    """nslab > 1 where the split solve does not apply (the reference's m =
    50, not a multiple of 128; the literal dot order; condtype 2's CSR
    operator): a warning on stderr and the one-context solve -- the same
    output as nslab = 1, not an abort"""
    prog = exe("bondc", 0)
    out = {}
    m = 50 if not extra else 128
    for k in (1, 2):
        d = tmp_path / ("k%d" % k)
        d.mkdir()
        (d / "bondc.nml").write_text("&bondc_nml lattice=0, m=%d, n=60, pbc=0, pb=0.6, seed=626504, "
                                     "nslab=%d, xport=1%s /\n" % (m, k, (", " + extra) if extra else ""))
        r = subprocess.run([prog], cwd=d, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        assert ("solving on one context" in r.stderr) == (k > 1), r.stderr[-2000:]
        out[k] = ([l for l in r.stdout.splitlines() if "Conductance:" in l], (d / "bond.txt").read_bytes())
    assert out[1] == out[2]


@pytest.mark.gpu
def test_bondc_driver_random_conductances(tmp_path):
    """condtype = 2 (ConductCalc.m condtype 2 from the Fortran host:
    perc_set_conductcalc_weights): the driver's conductance equals the
    Python route's -- the same occupancy, the host replay's labels, the
    weights from numpy's MT19937 (api.conductcalc_weights), perc_set_bond_
    weights -- to the printed precision; and differs from the fixed-g0 run"""
    prog = exe("bondc", 0)
    m = n = 64
    got = {}
    for ct in (1, 2):
        d = tmp_path / ("c%d" % ct)
        d.mkdir()
        (d / "bondc.nml").write_text("&bondc_nml lattice=0, m=%d, n=%d, pbc=0, pb=0.6, seed=626504, "
                                     "tol=1e-13, itmax=100000, condtype=%d, cseed=1838534 /\n" % (m, n, ct))
        r = subprocess.run([prog], cwd=d, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [l for l in r.stdout.splitlines() if "Conductance:" in l][-1]
        got[ct] = [float(x) for x in line.split(":")[1].split()]
    nb = api.nbonds(0, m, n, 0)
    order = api.shuffled_ids(nb, 626504)
    b1, b2 = api.bond_list(0, m, n, 0)
    with api.Context(0, m, n, 0) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=int(0.6 * nb))
        assert ctx.label()["nspan"] > 0
        ln = ctx.label_numbers(PL.BOND)
        ctx.set_bond_weights(api.conductcalc_weights(PL.RULE_BOND, b1, b2, ln["bond_label"], None,
                                                     ln["perccln"]))
        c = ctx.conductance(tol=1e-13, itmax=100000)
    assert abs(got[2][0] - c["gtop"]) <= 1e-12 * abs(c["gtop"]), (got[2], c)
    assert abs(got[2][1] - c["gbot"]) <= 1e-12 * abs(c["gbot"]), (got[2], c)
    assert abs(got[2][0] - got[1][0]) > 1e-3 * abs(got[1][0])


@pytest.mark.gpu
@pytest.mark.parametrize("v", ["sq_bondc_p50", "sq_bondc_p60", "sq_bondc_20x30_p55", "sq_bondc_p60_pbc",
                               "tri_bondc_p35", "tri_bondc_p40_pbc"])
def test_bondc_driver_trace_log(v, tmp_path):
    """trace = 1 (with dot_order = 1, whose conductance line is the
    reference solver's bitwise): bondocc.txt -- every bond's step, the
    spanning test and the conductance, bondc.f:194-594 -- is the reference
    run's byte for byte (md5 of the reference's own file, tests/golden/*/
    meta.json)"""
    import hashlib
    md, r = run_variant(v, tmp_path, extra=["dot_order=1", "trace=1"])
    got = hashlib.md5((tmp_path / "bondocc.txt").read_bytes()).hexdigest()
    assert got == md["files"]["bondocc.txt"], v


TRACE_LOGS = [(v, f) for v in G.variants() for f in ("siteocc.txt", "sbdebug.txt", "bsdebug.txt")
              if f in G.meta(v).get("files", {})]


@pytest.mark.parametrize("v,log", TRACE_LOGS)
def test_driver_trace_logs(v, log, tmp_path):
    """trace = 1: the per-step logs are the reference run's byte for byte
    (md5 of the reference's own file, tests/golden/*/meta.json) --
    siteocc.txt (site.f:167-350: each site's neighbours, largest neighbour
    cluster and absorbed clusters), sbdebug.txt (sitebond.f:184-465: the
    site phase, each bond's case with every site and bond a merge
    relabels) and bsdebug.txt (bondsite.f:178-418), each with its closing
    spanning test.  The drivers write them from the host replay before
    they open a device, so this runs with or without a GPU; with one (or
    for bondsite, which needs none) the run must also finish."""
    import hashlib
    md, r = run_variant(v, tmp_path, expect_ok=have_gpu() or md_kind(v) == "bondsite",
                        extra=["trace=1"])
    got = hashlib.md5((tmp_path / log).read_bytes()).hexdigest()
    assert got == md["files"][log], (v, log)
    if not have_gpu() and md_kind(v) != "bondsite":
        assert "status -8" in r.stderr


def md_kind(v):
    return G.meta(v)["kind"]


def test_replay_site_trace_records():
    """perc_replay_site_trace's records against the site replay: each
    step's joined cluster/size, and the absorbed sizes summing to the
    step's cluster size (lcs + sum(added) + 1)."""
    import numpy as np
    from percolation_amd import _lib as L
    lib = L.lib()
    m = n = 17
    order = np.random.default_rng(3).permutation(m * n).astype(np.int32) + 1
    k = int(0.7 * m * n)
    tr = np.zeros(24 * k, np.int32)
    assert lib.perc_replay_site_trace(0, m, n, 0, k, order.ctypes.data, tr.ctypes.data) == 0
    tr = tr.reshape(k, 24)
    assert (tr[:, 0] == order[:k]).all()
    for row in tr:
        if row[9] == 0:
            assert row[22] == 1 and row[10] == 0
        else:
            added = row[11:11 + 2 * row[10]:2]
            assert row[21] == row[8] and row[22] == row[9] + added.sum() + 1
    bad = order.copy()
    bad[0] = m * n + 1
    assert lib.perc_replay_site_trace(0, m, n, 0, k, bad.ctypes.data, np.zeros(24 * k, np.int32)
                                      .ctypes.data) == -7


def test_replay_mixed_trace_stream():
    """perc_replay_mixed_trace's stream parses into one record per step,
    its sizing call (trace = NULL) and a short buffer behave as declared,
    and a merge's relabelled sites are exactly the absorbed cluster's
    (checked against the replay's final labels: they all end in lcn's
    cluster unless a later merge moved it)."""
    import ctypes as C
    import numpy as np
    lib = PL.lib()
    m = n = 12
    t = m * n
    nb = lib.perc_nbonds(0, m, n, 0)
    rng = np.random.default_rng(5)
    so = (rng.permutation(t) + 1).astype(np.int32)
    bo = (rng.permutation(nb) + 1).astype(np.int32)
    ts, tb = int(0.6 * t), int(0.6 * nb)
    for kind, steps in ((PL.SITEBOND, tb), (PL.BONDSITE, ts)):
        ln = C.c_longlong(0)
        assert lib.perc_replay_mixed_trace(0, m, n, 0, kind, ts, so.ctypes.data, tb, bo.ctypes.data,
                                           None, 0, C.byref(ln)) == 0
        assert ln.value > steps
        ev = np.zeros(ln.value, np.int32)
        assert lib.perc_replay_mixed_trace(0, m, n, 0, kind, ts, so.ctypes.data, tb, bo.ctypes.data,
                                           ev.ctypes.data, ln.value - 1, C.byref(ln)) == -1
        assert lib.perc_replay_mixed_trace(0, m, n, 0, kind, ts, so.ctypes.data, tb, bo.ctypes.data,
                                           ev.ctypes.data, ln.value, C.byref(ln)) == 0
        r, recs, merges = 0, 0, 0
        while r < len(ev):
            e = ev[r]
            if kind == PL.BONDSITE:
                r += 2 if e == 0 else 4 + 2 * ev[r + 1]
            elif e == 0:
                r += 2
            elif e in (1, 2):
                r += 4
            elif e == 3:
                r += 8
            elif e in (4, 5):
                k = r + 7
                ns = ev[k]
                sites = ev[k + 1:k + 1 + ns]
                assert ns >= 1 and (np.diff(sites) > 0).all()
                k += 1 + ns
                k += 1 + ev[k]
                lcn, size, old = ev[k:k + 3]
                assert old != lcn and size >= ns + 2
                merges += 1
                r = k + 3
            else:
                assert e == 6
                r += 1
            recs += 1
        assert r == len(ev) and recs == steps
        if kind == PL.SITEBOND:
            assert merges > 0
