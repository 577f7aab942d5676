"""CPU-side checks of libperc's host logic (no device needed).

* the C-ABI library loads and exports every symbol include/perc.h declares;
* RNG, nearestn, bond list, REAL*4 shuffle equal the oracle (itself pinned
  to the reference);
* the host label replay reproduces the reference's bond.txt / site.txt /
  sbsite.txt / sbbond.txt byte-for-byte and the oracle's literal O(N^2)
  labeling on further seeds / sizes / lattices.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import golden_io as G
import oracle_lib as O
import percolation_amd as P
from percolation_amd import _lib as PL
from percolation_amd import api

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    hdr = open(os.path.join(REPO, "include", "perc.h")).read()
    return re.findall(r"^(?:void|int|float|double|const char)\s*\*?\s*(\w+)\s*\(", hdr, re.M)


def test_exports_every_declared_symbol():
    names = header_symbols()
    assert len(names) >= 25
    lib = C.CDLL(PL.LIBPERC)
    for n in names:
        assert hasattr(lib, n), n
        assert n in PL.SIGNATURES, n
    P.lib()  # signatures bind


_RUNTIMES_PROBE = """
import re, sys
sys.path.insert(0, %r)
from percolation_amd import _lib as PL
PL.lib()
try:
    import torch  # after libperc: the order that used to load a second runtime
    print("torch imported", flush=True)
except PL.PercError as e:
    print("refused:", e, flush=True)
maps = open('/proc/self/maps').read()
print(sorted(set(re.findall(r'(/\\S*(?:libamdhip64|libhsa-runtime64|librccl)\\S*)', maps))))
"""


@pytest.mark.parametrize("no_torch", [False, True])
def test_one_hip_runtime_per_process(no_torch):
    """libperc loaded before torch must not leave two HIP / HSA / RCCL
    runtimes in the process: that was round 4's interpreter-teardown abort
    (glibc "double free or corruption (!prev)", SIGABRT).  _lib.lib()
    imports torch first, so the default run has torch's copies alone; with
    PERC_NO_TORCH=1 libperc binds /opt/rocm's copies, and the later `import
    torch` is REFUSED with PercError before torch's libraries load (the
    runtime guard, _lib._SecondRuntimeGuard): still one runtime, exit 0"""
    import subprocess
    import sys
    pytest.importorskip("torch")
    env = dict(os.environ)
    env.pop("PERC_NO_TORCH", None)
    if no_torch:
        env["PERC_NO_TORCH"] = "1"
    r = subprocess.run([sys.executable, "-c", _RUNTIMES_PROBE % REPO], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    libs = eval(r.stdout.strip().splitlines()[-1])
    hip = [x for x in libs if "libamdhip64" in x]
    assert len(hip) == 1, libs
    if no_torch:
        assert "refused: import torch after libperc would load a second HIP runtime" in r.stdout, r.stdout
        assert "/opt/rocm" in hip[0], hip
    else:
        assert "torch imported" in r.stdout and len(libs) == 3, (r.stdout, libs)


_SECOND_RUNTIME_PROBE = """
import ctypes as C, sys
sys.path.insert(0, %r)
from percolation_amd import _lib as PL
L = PL.lib()                      # PERC_NO_TORCH=1: /opt/rocm's runtime
C.CDLL(%r, mode=C.RTLD_LOCAL)     # a second copy mapped behind libperc's back
n, paths = PL.runtimes()
h = C.c_void_p()
rc = L.perc_ctx_create(0, 0, 16, 16, 0, C.byref(h))
print(n, rc, L.perc_last_error().decode(), flush=True)
"""


def test_second_runtime_is_refused_by_the_library():
    """The C-ABI's own check (perc_hip_runtimes, perc_ctx_create): with a
    second libamdhip64 mapped in the process -- whatever loaded it -- the
    context is refused with PERC_ESTATE naming both copies, before any HIP
    call (a Fortran or C caller gets the same status).  The child's exit
    status is not checked: two runtimes may corrupt the heap at teardown,
    which is the condition being refused."""
    import subprocess
    import sys
    torch_rt = PL._torch_runtime()
    if not torch_rt:
        pytest.skip("no bundled runtime to map")
    env = dict(os.environ, PERC_NO_TORCH="1")
    r = subprocess.run([sys.executable, "-c", _SECOND_RUNTIME_PROBE % (REPO, torch_rt)],
                       capture_output=True, text=True, timeout=300, env=env)
    line = [x for x in r.stdout.splitlines() if x[:2] == "2 "]
    assert line, (r.stdout, r.stderr[-2000:])
    n, rc, msg = line[0].split(" ", 2)
    assert int(rc) == -9 and "two HIP runtimes" in msg and torch_rt in msg, line


def test_no_device_is_an_error_not_a_fallback():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("device present")
    except ImportError:
        pass
    h = C.c_void_p()
    rc = P.lib().perc_ctx_create(0, 0, 16, 16, 0, C.byref(h))
    assert rc == -8  # PERC_ENODEV


def test_rng_equals_oracle():
    L, Or = P.lib(), O.lib()
    for seed in (626504, 62703, 0, 1, 58302, 2147483646):
        L.perc_srand(seed)
        Or.or_srand(seed)
        a = np.array([L.perc_rand(0) for _ in range(5000)], np.float32)
        b = np.array([Or.or_rand(0) for _ in range(5000)], np.float32)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(api.trial_seeds(58302, 1000), _oracle_seeds(58302))


def _oracle_seeds(master):
    ts = O.i32(1000)
    O.lib().or_trial_seeds(master, 1000, ts)
    return ts


LATTICES = [(0, 50, 50, 0), (0, 50, 50, 1), (1, 50, 50, 0), (1, 50, 50, 1), (0, 7, 9, 0),
            (0, 7, 9, 1), (1, 8, 6, 1), (1, 10, 10, 0), (0, 3, 3, 0)]


@pytest.mark.parametrize("lat,m,n,pbc", LATTICES)
def test_topology_equals_oracle(lat, m, n, pbc):
    nn_o = O.i32(6)
    for rn in range(1, m * n + 1):
        O.lib().or_nearestn(lat, m, n, pbc, rn, nn_o)
        scn = 6 if lat else 4
        assert list(api.nearestn(lat, m, n, pbc, rn)) == list(nn_o[:scn]), rn
    b1, b2 = api.bond_list(lat, m, n, pbc)
    ob1, ob2 = O.bond_list(lat, m, n, pbc)
    assert np.array_equal(b1, ob1) and np.array_equal(b2, ob2)


@pytest.mark.parametrize("lat,m,n,pbc", [l for l in LATTICES if not (l[0] == 1 and l[1] % 2)])
def test_neighbour_relation_symmetric(lat, m, n, pbc):
    """Even-m lattices (all configs) have a symmetric nearestn relation;
    libperc relies on it (odd-m triangular is rejected: hazard H7)."""
    t = m * n
    adj = {rn: set(int(x) for x in api.nearestn(lat, m, n, pbc, rn) if x) for rn in range(1, t + 1)}
    for a, ns in adj.items():
        for b in ns:
            assert a in adj[b], (a, b)


@pytest.mark.parametrize("v", [v for v in G.variants() if G.meta(v)["kind"] == "bondc"])
def test_shuffle_reproduces_bondorder(v):
    p = G.meta(v)["params"]
    b1, b2 = api.bond_list(p["lattice"], p["m"], p["n"], p["pbc"])
    order = api.shuffled_ids(len(b1), p["seed"])[:len(b1)]
    o1 = np.where(order > 0, b1[order - 1], 0)
    o2 = np.where(order > 0, b2[order - 1], 0)
    assert G.fmt_i10(o1, o2) == G.text(v, "bondorder.txt")


@pytest.mark.parametrize("v", [v for v in G.variants() if G.meta(v)["kind"] == "bondc"])
def test_replay_bond_txt(v):
    md = G.meta(v)
    p = md["params"]
    nb = api.nbonds(p["lattice"], p["m"], p["n"], p["pbc"])
    b1, b2 = api.bond_list(p["lattice"], p["m"], p["n"], p["pbc"])
    order = api.shuffled_ids(nb, p["seed"])
    tb = int(p["pb"] * nb)
    r = api.replay_labels(p["lattice"], p["m"], p["n"], p["pbc"], PL.BOND, bond_order=order,
                          nbond=tb)
    txt = api.fmt_i10(b1, b2, r["bond_label"], np.arange(1, nb + 1), r["csize"][1:nb + 1])
    assert txt.encode() == G.text(v, "bond.txt")
    assert r["perccln"] == md["perccln"]
    assert (r["maxcn"], r["maxcs"]) == (md["maxcn"], md["maxcs"])


@pytest.mark.parametrize("v", [v for v in G.variants() if G.meta(v)["kind"] == "site"])
def test_replay_site_txt(v):
    md = G.meta(v)
    p = md["params"]
    t = p["m"] * p["n"]
    order = api.shuffled_ids(t, p["seed"])
    assert "".join(" %d\n" % x for x in order[:t]).encode() == G.text(v, "siteorder.txt")
    ts = int(p["ps"] * t)
    r = api.replay_labels(p["lattice"], p["m"], p["n"], p["pbc"], PL.SITE, site_order=order,
                          nsites=ts)
    txt = api.fmt_i10(np.arange(1, t + 1), r["site_label"], r["csize"][1:t + 1])
    assert txt.encode() == G.text(v, "site.txt")
    assert r["perccln"] == md["perccln"]
    assert (r["maxcn"], r["maxcs"]) == (md["maxcn"], md["maxcs"])


@pytest.mark.parametrize("v", [v for v in G.variants() if G.meta(v)["kind"] == "sitebond"])
def test_replay_sitebond_txt(v):
    md = G.meta(v)
    p = md["params"]
    lat, m, n, pbc = p["lattice"], p["m"], p["n"], p["pbc"]
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    b1, b2 = api.bond_list(lat, m, n, pbc)
    so = api.shuffled_ids(t, p["sseed"])
    bo = api.shuffled_ids(nb, p["bseed"])
    r = api.replay_labels(lat, m, n, pbc, PL.SITEBOND, site_order=so, nsites=int(p["ps"] * t),
                          bond_order=bo, nbond=int(p["pb"] * nb))
    assert api.fmt_i10(np.arange(1, t + 1), r["site_label"],
                       r["csize"][1:t + 1]).encode() == G.text(v, "sbsite.txt")
    assert api.fmt_i10(b1, b2, r["bond_label"]).encode() == G.text(v, "sbbond.txt")
    assert r["perccln"] == md["perccln"]
    assert (r["maxcn"], r["maxcs"]) == (md["maxcn"], md["maxcs"])


CASES = [(0, 30, 40, 0, 0.5, 11), (0, 30, 40, 1, 0.55, 12), (1, 30, 40, 0, 0.35, 13),
         (1, 30, 40, 1, 0.40, 14), (0, 64, 64, 0, 0.5, 15), (0, 33, 21, 0, 0.62, 16)]


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES)
def test_replay_equals_literal_bonds(lat, m, n, pbc, p, seed):
    b1, b2, o1, o2 = O.bond_order(lat, m, n, pbc, seed)
    nb = len(b1)
    tb = int(p * nb)
    lab, cs, cln, mx, ms = O.label_bonds(lat, m, n, pbc, b1, b2, o1, o2, tb, literal=True)
    order = api.shuffled_ids(nb, seed)
    r = api.replay_labels(lat, m, n, pbc, PL.BOND, bond_order=order, nbond=tb)
    assert np.array_equal(r["bond_label"], lab)
    assert np.array_equal(r["csize"][:nb + 2], cs)
    assert (r["cln"], r["maxcn"], r["maxcs"]) == (cln, mx, ms)


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES)
def test_replay_equals_literal_sites(lat, m, n, pbc, p, seed):
    t = m * n
    order = O.site_order(t, seed)
    ts = int((p + 0.1) * t)
    s, cs, cln, mx, ms = O.label_sites(lat, m, n, pbc, order, ts, literal=True)
    r = api.replay_labels(lat, m, n, pbc, PL.SITE, site_order=api.shuffled_ids(t, seed),
                          nsites=ts)
    assert np.array_equal(r["site_label"], s)
    assert np.array_equal(r["csize"][:t + 2], cs)
    assert (r["cln"], r["maxcn"], r["maxcs"]) == (cln, mx, ms)


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES[:4])
def test_replay_equals_literal_sitebond(lat, m, n, pbc, p, seed):
    t = m * n
    Or = O.lib()
    so = O.site_order(t, seed)
    b1, b2, o1, o2 = O.bond_order(lat, m, n, pbc, seed + 100)
    nb = len(b1)
    ts, tb = int(0.7 * t), int(p * nb)
    s, bl, cs = O.i32(t), O.i32(nb), O.i32(t + nb + 2)
    mx, ms = C.c_int(), C.c_int()
    cln = Or.or_label_sitebond(lat, m, n, pbc, nb, b1, b2, so, ts, o1, o2, tb, s, bl, cs,
                               C.byref(mx), C.byref(ms))
    r = api.replay_labels(lat, m, n, pbc, PL.SITEBOND, site_order=api.shuffled_ids(t, seed),
                          nsites=ts, bond_order=api.shuffled_ids(nb, seed + 100), nbond=tb)
    assert np.array_equal(r["site_label"], s)
    assert np.array_equal(r["bond_label"], bl)
    assert np.array_equal(r["csize"], cs)
    assert (r["cln"], r["maxcn"], r["maxcs"]) == (cln, mx.value, ms.value)


@pytest.mark.parametrize("lat,m,n,pbc,p,seed", CASES)
@pytest.mark.parametrize("ps", [0.45, 0.8])
def test_replay_equals_literal_bondsite(lat, m, n, pbc, p, seed, ps):
    """PERC_BONDSITE replay (union-find) == the oracle's literal bondsite.f
    loops: labels, sizes, cln, largest cluster, spanning label."""
    t = m * n
    Or = O.lib()
    b1, b2 = O.bond_list(lat, m, n, pbc)
    nb = len(b1)
    so, bo = O.site_order(t, seed), O.site_order(nb, seed + 100)
    ts, tb = int(ps * t), int(p * nb)
    s, bl, cs = O.i32(t), O.i32(nb), O.i32(t + nb + 2)
    mx, ms = C.c_int(), C.c_int()
    cln = Or.or_label_bondsite(lat, m, n, pbc, nb, b1, b2, bo, tb, so, ts, s, bl, cs,
                               C.byref(mx), C.byref(ms))
    r = api.replay_labels(lat, m, n, pbc, PL.BONDSITE, site_order=api.shuffled_ids(t, seed),
                          nsites=ts, bond_order=api.shuffled_ids(nb, seed + 100), nbond=tb)
    assert np.array_equal(r["site_label"], s)
    assert np.array_equal(r["bond_label"], bl)
    assert np.array_equal(r["csize"], cs)
    assert (r["cln"], r["maxcn"], r["maxcs"]) == (cln, mx.value, ms.value)
    assert r["perccln"] == Or.or_span_sites(m, n, s, cs, cln, 2 * n - 1)


def test_pb_grid_matches_reference_rows():
    """nbarr of bond_cond.f:84-97 gives the reference's row pb values."""
    for v in [v for v in G.variants() if G.meta(v)["kind"] == "bond_cond"]:
        p = G.meta(v)["params"]
        nb = api.nbonds(p["lattice"], p["m"], p["n"], p["pbc"])
        nbarr = api.pb_grid(p["lattice"], nb)
        rows = [l for l in G.text(v, "bondcond.txt").decode().splitlines() if l.count(",") == 3]
        first_trial = []
        for l in rows:
            pbv = float(l.split(",")[0])
            if first_trial and pbv <= first_trial[-1]:
                break
            first_trial.append(pbv)
        want = []
        for k, bf in enumerate(nbarr):
            if bf <= 0 or (want and bf <= want[-1][0]):
                break
            want.append((bf, float(np.float32(np.float32(bf) / np.float32(nb)))))
        assert ["%11.9f" % x for _, x in want] == ["%11.9f" % x for x in first_trial]


def test_degenerate_lattice_is_rejected():
    """m or n below 3 (no interior row or column to solve for) is refused
    with PERC_EINVAL, before any device is touched."""
    for m, n in [(2, 3), (3, 2), (1, 1)]:
        with pytest.raises(P.PercError, match="PERC_EINVAL"):
            api.Context(0, m, n, 0)


def test_random_order_is_a_keyed_permutation():
    """perc_random_order (the order perc_occupy_random's occupancy is a
    prefix of): a permutation of 1..n, every prefix the prefix of the full
    order, deterministic in the seed, the bond stream distinct from the site
    stream, and roughly uniform (prefix means)."""
    import numpy as np
    from percolation_amd import _lib as PL
    n = 5000
    full = api.random_order(n, n, 7)
    assert sorted(full.tolist()) == list(range(1, n + 1))
    for c in (0, 1, 17, 2500, n):
        assert np.array_equal(api.random_order(n, c, 7), full[:c])
    assert np.array_equal(api.random_order(n, n, 7), full)
    assert not np.array_equal(api.random_order(n, 100, 8), full[:100])
    assert not np.array_equal(api.random_order(n, 100, 7, PL.SITE), full[:100])
    means = [api.random_order(n, 1000, s_).mean() for s_ in range(20)]
    assert abs(np.mean(means) - (n + 1) / 2) < 0.05 * n


def test_random_order_keys_are_the_defined_hash():
    """The occupancy draw's keys, computed in 32-bit arithmetic with the seed
    folded in once (lattice.h perc_rand_hash32, the device kernels' and the
    host order's arithmetic), are the documented definition
    (perc_rand_key: hash32 = high word of splitmix64(splitmix64(seed) ^ id),
    key = hash32 << 32 | id; the bond stream seeded by
    splitmix64(seed ^ 0x5DEECE66D)) -- restated here in Python integers."""
    from percolation_amd import _lib as PL
    M = (1 << 64) - 1

    def mix64(x):
        x = (x + 0x9E3779B97F4A7C15) & M
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
        return x ^ (x >> 31)

    n = 3000
    for seed in (0, 1, 58302, 0xFFFFFFFF, 0x123456789ABCDEF0, M):
        for kind, s_ in ((PL.SITE, seed), (PL.BOND, mix64(seed ^ 0x5DEECE66D))):
            S = mix64(s_)
            want = sorted(range(1, n + 1), key=lambda i: ((mix64(S ^ i) >> 32) << 32) | i)
            assert api.random_order(n, n, seed, kind).tolist() == want, (seed, kind)


@pytest.mark.parametrize("m,n,pbc", [(5, 4, 0), (5, 4, 1), (64, 33, 0), (17, 40, 1), (2, 3, 1)])
def test_square_bond_first_closed_form(m, n, pbc):
    """lattice.h bf_square: bond_first of the square lattice's rows 0..n-2 is
    r*(2m-1+pbc) + 2c + pbc*(c>0) -- the form k_assemble / k_cc_tile use when
    the context's built bond_first agrees (perc_ctx::bf_closed)."""
    b1, b2 = api.bond_list(0, m, n, pbc)
    lo = np.minimum(b1, b2)
    counts = np.bincount(lo, minlength=m * n + 2)
    first = np.concatenate([[0], np.cumsum(counts)])  # first[s] = bonds with smaller end < s
    for r in range(n - 1):
        for c in range(m):
            assert first[r * m + c + 1] == r * (2 * m - 1 + pbc) + 2 * c + (pbc if c > 0 else 0)


@pytest.mark.parametrize("seed", [0, 1, 1838534, 2 ** 32 - 1])
def test_twister_equals_numpy_mt19937(seed):
    """perc_twister_uniform (the C generator behind perc_set_conductcalc_
    weights, ConductCalc.m:38-47 rand('twister', seed)) draws numpy's
    RandomState(seed).random_sample bitwise: MT19937 init_genrand + 53-bit
    genrand_res53, over several state refills"""
    got = api.twister_uniform(seed, 3000)
    want = np.random.RandomState(seed).random_sample(3000)
    assert np.array_equal(got, want)
