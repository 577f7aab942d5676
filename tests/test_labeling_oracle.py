"""GPU labeling against the oracle's own replays, directly (no libperc replay
in between), over block-edge geometries and at the BASELINE config sizes.

The GPU labels with an LDS-tiled union-find (k_cc_tile over 128 x 32 blocks
of sites, k_cc_merge for the links that cross a block edge, k_cc_compress):
the partition (canonical id = minimum site of the cluster) must equal the
partition of the reference's sequential labeling (Square/bondc.f:194-393,
site.f:167-289, sitebond.f:187-400) bit for bit, and a spanning cluster must
be found exactly when the reference finds one (bondc.f:413-456,
site.f:309-344, sitebond.f:423-458).  The oracle side is oracle/perc_oracle.c
(O(N alpha) replays; the mixed replay is pinned to the literal loop here on
CPU).
"""
import numpy as np
import pytest

import oracle_lib as O
from percolation_amd import _lib as PL
from percolation_amd import api


def _perm_ids(N, seed):
    """uniform 1-based id permutation (the bench's occupation orders)"""
    return (np.random.default_rng(seed).permutation(N) + 1).astype(np.int32)


def _pairs(b1, b2, ids, k):
    o1, o2 = O.i32(len(b1) + 1), O.i32(len(b1) + 1)
    sel = ids[:k].astype(np.int64) - 1
    o1[:k], o2[:k] = b1[sel], b2[sel]
    return o1, o2


def oracle_bond(lat, m, n, pbc, ids, tb):
    b1, b2 = O.bond_list(lat, m, n, pbc)
    o1, o2 = _pairs(b1, b2, ids, tb)
    label, csize, cln, _, _ = O.label_bonds(lat, m, n, pbc, b1, b2, o1, o2, tb, literal=False)
    perccln = O.lib().or_span_bonds(m, n, len(b1), b1, b2, label, csize, cln)
    canon = O.canon_bonds(m * n, b1, b2, label, cln)
    span_root = 0
    if perccln > 0:
        k = int(np.nonzero(label == perccln)[0][0])
        span_root = int(canon[b1[k] - 1])
    return canon, perccln, span_root


def oracle_site(lat, m, n, pbc, order, ts):
    o = O.i32(m * n + 1)
    o[:len(order)] = order
    s, csize, cln, _, _ = O.label_sites(lat, m, n, pbc, o, ts, literal=False)
    perccln = O.lib().or_span_sites(m, n, s, csize, cln, n)
    canon = O.canon_sites(s, cln)
    span_root = int(canon[np.nonzero(s == perccln)[0][0]]) if perccln > 0 else 0
    return canon, perccln, span_root


def oracle_mixed(lat, m, n, pbc, sids, ts, bids, tb):
    b1, b2 = O.bond_list(lat, m, n, pbc)
    so = O.i32(m * n + 1)
    so[:len(sids)] = sids
    o1, o2 = _pairs(b1, b2, bids, tb)
    s, bl, csize, cln, _, _ = O.label_sitebond(lat, m, n, pbc, b1, b2, so, ts, o1, o2, tb,
                                               literal=False)
    perccln = O.lib().or_span_sites(m, n, s, csize, cln, 2 * n - 1)
    # the site partition: only sites carry the spanning test and the
    # ConductCalc mixed rule; bonds with both ends empty form clusters of
    # their own that no site belongs to
    canon = O.canon_sites(s, cln)
    span_root = int(canon[np.nonzero(s == perccln)[0][0]]) if perccln > 0 else 0
    return canon, perccln, span_root


def gpu_label(lat, m, n, pbc, kind, sids=None, ts=0, bids=None, tb=0):
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(kind, site_order=sids, nsites=ts, bond_order=bids, nbonds_=tb)
        return ctx.label(canon=True)


def check(li, canon, perccln, span_root):
    got = li["canon"]
    if not np.array_equal(got, canon):
        bad = np.nonzero(got != canon)[0]
        raise AssertionError("partition differs at %d sites, first site %d: gpu %d oracle %d"
                             % (len(bad), bad[0] + 1, got[bad[0]], canon[bad[0]]))
    assert (li["nspan"] > 0) == (perccln > 0), (li["nspan"], perccln)
    if perccln > 0:
        assert li["span_root"] == span_root
    # the cluster count (a pass over the member roots, or -- the site and
    # mixed kinds on the open square lattice -- the wave tiles' member roots
    # minus the merge's hooks) is the partition's
    assert li["nclusters"] == len(np.unique(canon[canon > 0])), (li["nclusters"], len(np.unique(canon[canon > 0])))


# ------------------------------------------------------------ CPU: the oracle's mixed replay
@pytest.mark.parametrize("lat,m,n,pbc,ps,pb,seed", [
    (0, 20, 20, 0, 0.6, 0.5, 1), (0, 24, 18, 1, 0.8, 0.7, 2), (1, 20, 16, 0, 0.7, 0.6, 3),
    (1, 22, 20, 1, 0.9, 0.4, 4), (0, 30, 30, 0, 0.593, 1.0, 5), (1, 18, 18, 0, 1.0, 0.5, 6)])
def test_sitebond_replay_equals_literal(lat, m, n, pbc, ps, pb, seed):
    t = m * n
    b1, b2, o1, o2 = O.bond_order(lat, m, n, pbc, seed)
    so = O.site_order(t, seed + 100)
    ts, tb = int(ps * t), int(pb * len(b1))
    lit = O.label_sitebond(lat, m, n, pbc, b1, b2, so, ts, o1, o2, tb, literal=True)
    rep = O.label_sitebond(lat, m, n, pbc, b1, b2, so, ts, o1, o2, tb, literal=False)
    for a, b in zip(lit[:3], rep[:3]):
        assert np.array_equal(a, b)
    assert lit[3:] == rep[3:]


def test_canon_helpers_match_python():
    lat, m, n, pbc = 0, 40, 30, 0
    b1, b2, o1, o2 = O.bond_order(lat, m, n, pbc, 77)
    tb = len(b1) // 2
    label, _, cln, _, _ = O.label_bonds(lat, m, n, pbc, b1, b2, o1, o2, tb, literal=False)
    want = np.zeros(m * n, np.int64)
    for lab in np.unique(label[label > 0]):
        ks = np.nonzero(label == lab)[0]
        sites = np.concatenate([b1[ks], b2[ks]])
        want[sites - 1] = sites.min()
    assert np.array_equal(O.canon_bonds(m * n, b1, b2, label, cln), want)
    so = O.site_order(m * n, 5)
    s, _, cln, _, _ = O.label_sites(lat, m, n, pbc, so, 700, literal=False)
    want = np.zeros(m * n, np.int64)
    for lab in np.unique(s[s > 0]):
        idx = np.nonzero(s == lab)[0]
        want[idx] = idx.min() + 1
    assert np.array_equal(O.canon_sites(s, cln), want)


# ------------------------------------------------------------ GPU: block-edge geometries
# widths / heights that are not multiples of the 128 x 32 block, pbc wraps,
# triangular diagonals across block edges, single block rows
GEOMS = [(0, 200, 70, 0), (0, 384, 65, 1), (0, 129, 31, 1), (1, 130, 33, 0), (1, 256, 96, 1),
         (1, 64, 40, 1), (0, 1000, 33, 1), (0, 16, 300, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("p", [0.45, 0.6, 0.9])
def test_bond_partition_vs_oracle(geom, p):
    lat, m, n, pbc = geom
    nb = api.nbonds(lat, m, n, pbc)
    ids = api.shuffled_ids(nb, 1000 + m + n)
    if lat == 1:
        p -= 0.12
    tb = int(p * nb)
    li = gpu_label(lat, m, n, pbc, PL.BOND, bids=ids, tb=tb)
    check(li, *oracle_bond(lat, m, n, pbc, ids, tb))


@pytest.mark.gpu
@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("p", [0.45, 0.6, 0.9])
def test_site_partition_vs_oracle(geom, p):
    lat, m, n, pbc = geom
    t = m * n
    ids = api.shuffled_ids(t, 2000 + m + n)
    ts = int(p * t)
    li = gpu_label(lat, m, n, pbc, PL.SITE, sids=ids, ts=ts)
    check(li, *oracle_site(lat, m, n, pbc, ids, ts))


@pytest.mark.gpu
@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("ps,pb", [(0.6, 0.9), (0.85, 0.85), (1.0, 0.5)])
def test_mixed_partition_vs_oracle(geom, ps, pb):
    lat, m, n, pbc = geom
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    sids, bids = api.shuffled_ids(t, 3000 + m), api.shuffled_ids(nb, 4000 + n)
    ts, tb = int(ps * t), int(pb * nb)
    li = gpu_label(lat, m, n, pbc, PL.SITEBOND, sids=sids, ts=ts, bids=bids, tb=tb)
    check(li, *oracle_mixed(lat, m, n, pbc, sids, ts, bids, tb))


# ------------------------------------------------------------ GPU: the open square lattice's wave tiles
# (k_cc_tile_w: 128 x 16 blocks, ballot masks for site / mixed; k_cc_merge_sq)
# at widths and heights on either side of the block edges, near each kind's
# threshold and far above it
SQ_OPEN = [(127, 15), (128, 16), (129, 17), (255, 31), (257, 33), (384, 100), (513, 47), (64, 129),
           (3, 40), (300, 3), (130, 4)]


@pytest.mark.gpu
@pytest.mark.parametrize("m,n", SQ_OPEN)
@pytest.mark.parametrize("kind", [PL.BOND, PL.SITE, PL.SITEBOND])
def test_open_square_block_edges_vs_oracle(m, n, kind):
    t, nb = m * n, api.nbonds(0, m, n, 0)
    rng = np.random.default_rng(m * 1000 + n + kind)
    for p in (rng.uniform(0.45, 0.55), rng.uniform(0.6, 0.75), 0.95):
        if kind == PL.BOND:
            ids = _perm_ids(nb, int(rng.integers(1 << 30)))
            tb = int(p * nb)
            li = gpu_label(0, m, n, 0, PL.BOND, bids=ids, tb=tb)
            check(li, *oracle_bond(0, m, n, 0, ids, tb))
        elif kind == PL.SITE:
            ids = _perm_ids(t, int(rng.integers(1 << 30)))
            ts = int((p + 0.1 if p < 0.9 else p) * t)
            li = gpu_label(0, m, n, 0, PL.SITE, sids=ids, ts=min(ts, t))
            check(li, *oracle_site(0, m, n, 0, ids, min(ts, t)))
        else:
            sids = _perm_ids(t, int(rng.integers(1 << 30)))
            bids = _perm_ids(nb, int(rng.integers(1 << 30)))
            ts, tb = int(min(p + 0.15, 1.0) * t), int(min(p + 0.1, 1.0) * nb)
            li = gpu_label(0, m, n, 0, PL.SITEBOND, sids=sids, ts=ts, bids=bids, tb=tb)
            check(li, *oracle_mixed(0, m, n, 0, sids, ts, bids, tb))


# ------------------------------------------------------------ GPU: BASELINE config sizes
@pytest.mark.gpu
def test_metric_bond_4096_partition_vs_oracle():
    """the metric workload's partition (square 4096^2, bond p = 0.6, the
    bench's uniform order of its first realisation)"""
    lat, m, n, pbc = 0, 4096, 4096, 0
    nb = api.nbonds(lat, m, n, pbc)
    seed = int(api.trial_seeds(58302, 1)[0])
    ids = _perm_ids(nb, seed)
    tb = int(0.6 * nb)
    li = gpu_label(lat, m, n, pbc, PL.BOND, bids=ids, tb=tb)
    check(li, *oracle_bond(lat, m, n, pbc, ids, tb))
    assert li["nspan"] == 1


@pytest.mark.gpu
def test_config3_tri_site_1024_partition_vs_oracle():
    """config 3: triangular 1024^2 site p = 0.5, reference shuffle of tseed(1)"""
    lat, m, n, pbc = 1, 1024, 1024, 0
    t = m * n
    ids = api.shuffled_ids(t, int(api.trial_seeds(58302, 1)[0]))
    ts = t // 2
    li = gpu_label(lat, m, n, pbc, PL.SITE, sids=ids, ts=ts)
    check(li, *oracle_site(lat, m, n, pbc, ids, ts))


@pytest.mark.gpu
@pytest.mark.parametrize("ps,pb", [(0.593, 0.50), (0.85, 0.85)])
def test_config5_mixed_8192_partition_vs_oracle(ps, pb):
    """config 5: square 8192^2 mixed site-then-bond at ps = 0.593, pb = 0.5
    (sub-critical under the reference rule) and its
    near-critical companion; uniform orders"""
    lat, m, n, pbc = 0, 8192, 8192, 0
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    sids, bids = _perm_ids(t, 8192), _perm_ids(nb, 8193)
    ts, tb = int(ps * t), int(pb * nb)
    li = gpu_label(lat, m, n, pbc, PL.SITEBOND, sids=sids, ts=ts, bids=bids, tb=tb)
    check(li, *oracle_mixed(lat, m, n, pbc, sids, ts, bids, tb))


# ------------------------------------------------------------ GPU: device-drawn occupancy
@pytest.mark.gpu
@pytest.mark.parametrize("lat,m,n,pbc", [(0, 200, 70, 0), (1, 130, 90, 1), (0, 512, 512, 0)])
@pytest.mark.parametrize("kind", [PL.BOND, PL.SITE, PL.SITEBOND])
def test_occupy_random_equals_its_host_order(lat, m, n, pbc, kind):
    """perc_occupy_random (keys + radix select on the GPU) occupies exactly
    the prefix of perc_random_order (host): same partition as occupying that
    order explicitly, the same reference label numbers by replay (the host
    regenerates the order), and against the oracle's replay."""
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    ts, tb = int(0.62 * t), int(0.55 * nb)
    seed = 1234567 + m
    so = api.random_order(t, ts, seed, PL.SITE) if kind != PL.BOND else None
    bo = api.random_order(nb, tb, seed, PL.BOND) if kind != PL.SITE else None
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy_random(kind, ts if kind != PL.BOND else 0, tb if kind != PL.SITE else 0, seed)
        orr = ctx.occupancy()
        lr = ctx.label(canon=True)
        nr = ctx.label_numbers(kind)
        ctx.occupy(kind, site_order=so, nsites=ts if so is not None else 0, bond_order=bo,
                   nbonds_=tb if bo is not None else 0)
        ore = ctx.occupancy()
        le = ctx.label(canon=True)
        ne = ctx.label_numbers(kind)
    # the occupancy itself, element by element (sites and bonds)
    assert np.array_equal(orr[0], ore[0]) and np.array_equal(orr[1], ore[1])
    assert int(orr[0].sum()) == (ts if kind != PL.BOND else 0)
    assert int(orr[1].sum()) == (tb if kind != PL.SITE else 0)
    assert np.array_equal(lr["canon"], le["canon"])
    assert lr["nspan"] == le["nspan"] and lr["span_root"] == le["span_root"]
    for key in ("bond_label", "site_label"):
        if nr[key] is not None:
            assert np.array_equal(nr[key], ne[key])
    assert nr["perccln"] == ne["perccln"] and nr["maxcs"] == ne["maxcs"]
    if kind == PL.BOND:
        check(lr, *oracle_bond(lat, m, n, pbc, bo, tb))
    elif kind == PL.SITE:
        check(lr, *oracle_site(lat, m, n, pbc, so, ts))


@pytest.mark.gpu
@pytest.mark.parametrize("frac", [0.0, 1e-6, 0.003, 0.5, 0.997, 1.0])
@pytest.mark.parametrize("full", [False, True])
def test_occupy_random_select_extremes(frac, full, monkeypatch):
    """The on-device select (k_select_window + k_select_final) at the count
    extremes -- 1 element, a handful, almost all, n-1, n -- and with
    PERC_SELECT_FULL=1 (empty window: the exact all-keys path) occupies
    exactly the prefix of perc_random_order."""
    if full:
        monkeypatch.setenv("PERC_SELECT_FULL", "1")
    lat, m, n, pbc = 0, 300, 211, 0
    nb = api.nbonds(lat, m, n, pbc)
    for tb in sorted({max(1, int(frac * nb)), min(nb, max(1, int(frac * nb)) + 1), nb - 1}
                     if 0.0 < frac < 1.0 else ({1} if frac == 0.0 else {nb - 1, nb})):
        seed = 99 + tb
        bo = api.random_order(nb, tb, seed, PL.BOND)
        with api.Context(lat, m, n, pbc) as ctx:
            ctx.occupy_random(PL.BOND, 0, tb, seed)
            orr = ctx.occupancy()[1]
            lr = ctx.label(canon=True)
            ctx.occupy(PL.BOND, bond_order=bo, nbonds_=tb)
            ore = ctx.occupancy()[1]
            le = ctx.label(canon=True)
        assert np.array_equal(orr, ore) and int(orr.sum()) == tb, tb
        assert np.array_equal(lr["canon"], le["canon"]), tb
        assert lr["nspan"] == le["nspan"] and lr["nclusters"] == le["nclusters"], tb


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_bench_realisations_partition_vs_oracle(k):
    """The realisations bench.py times (L = 4096, bond p = 0.6, occupancy
    drawn on the GPU by perc_occupy_random with the seed tseed(k + 1) of
    master 58302, bond_cond.f:62-70): the GPU's partition of exactly that
    occupancy equals the oracle's replay of the same prefix of
    perc_random_order (Square/bondc.f:194-393), and so do the spanning
    verdict and root -- the timed workload itself, not a stand-in order."""
    lat, m, n, pbc = 0, 4096, 4096, 0
    nb = api.nbonds(lat, m, n, pbc)
    tb = int(0.6 * nb)
    seed = int(api.trial_seeds(58302, 1000)[k])
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy_random(PL.BOND, 0, tb, seed)
        li = ctx.label(canon=True)
    assert li["nspan"] > 0
    bo = api.random_order(nb, tb, seed, PL.BOND)
    check(li, *oracle_bond(lat, m, n, pbc, bo, tb))


@pytest.mark.gpu
@pytest.mark.parametrize("lat,m,n,pbc", [(0, 512, 512, 0), (0, 1000, 300, 0), (1, 256, 256, 0)])
@pytest.mark.parametrize("kind", [PL.BOND, PL.SITE, PL.SITEBOND])
def test_span_sites_with_and_without_the_speculative_count(lat, m, n, pbc, kind):
    """perc_label's span_sites (the spanning cluster's member sites): the
    first labeling of a context counts them after reading the spanning roots
    back; once a labeling has spanned, the next one flattens and counts on the
    device behind the spanning test (k_cc_compress_spec, one read-back) --
    both equal to the member sites whose canonical root is span_root, on
    realisations that span and ones that do not (a dense, a sparse, a dense
    draw in turn)."""
    t, nb = m * n, api.nbonds(lat, m, n, pbc)
    dense, sparse = 0.9, 0.2
    with api.Context(lat, m, n, pbc) as ctx:
        for k, f in enumerate((dense, dense, sparse, dense, dense)):
            ts = int(f * t) if kind != PL.BOND else 0
            tb = int(f * nb) if kind != PL.SITE else 0
            ctx.occupy_random(kind, ts, tb, 4242 + k)
            li = ctx.label()
            canon = ctx.label(canon=True)["canon"]  # (the same occupancy, labelled again)
            if li["nspan"] == 0:
                assert f == sparse
                continue
            assert f == dense and li["nspan"] == 1
            want = int(np.count_nonzero(canon == li["span_root"]))
            assert li["span_sites"] == want, (k, li["span_sites"], want)
