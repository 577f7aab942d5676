"""One conductance solve split over processes (percolation_amd/dslab.py,
perc_dslab_* in include/perc.h; SURVEY.md §8(f) row 2, the linbcg loop of
Square/bondc.f:780-836).

CPU: the exchange layer at world size 3 over gloo -- the all-gather puts
every slab's partials in slab order, and the halo swap hands slab s-1's
last row to slab s's lower ghost and slab s+1's first row to its upper
ghost.

GPU: K processes on the box's one GPU (gloo through host memory; RCCL
allows one rank per device) give perc_set_slabs(K)'s numbers in one process
bitwise -- same slab kernels, same slab-order combine; one process over
RCCL ("nccl", the multi-GPU transport) agrees with the single-slab solve
up to the dot association.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from percolation_amd import _lib as PL
from percolation_amd import api, dslab


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exchange_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = 5
        po = torch.arange(4, dtype=torch.float64) + 10 * rank
        pa = torch.zeros(4 * world, dtype=torch.float64)
        edges = tuple(torch.full((m,), 100.0 * rank + side, dtype=torch.float64)
                      if 0 <= rank + (2 * side - 1) < world else None for side in (0, 1))
        ghosts = tuple(torch.zeros(m, dtype=torch.float64) if e is not None else None for e in edges)
        ex = dslab._Exchange(None, world, rank, po, pa, edges, ghosts)
        ex.gather()
        ex.halo()
        q.put((rank, pa.tolist(), [None if g is None else g.tolist() for g in ghosts]))
    finally:
        dist.destroy_process_group()


def test_exchange_gather_and_halo_gloo():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.spawn(_exchange_worker, args=(world, free_port(), q), nprocs=world, join=True)
    got = {}
    while not q.empty():
        r, pa, gh = q.get()
        got[r] = (pa, gh)
    assert sorted(got) == [0, 1, 2]
    want = [v + 10 * r for r in range(world) for v in range(4)]
    for r in range(world):
        pa, (glo, ghi) = got[r]
        assert pa == want  # slab order on every process
        # lower ghost = slab r-1's upper edge (side 1), upper ghost = slab r+1's lower edge
        assert glo == (None if r == 0 else [100.0 * (r - 1) + 1] * 5)
        assert ghi == (None if r == world - 1 else [100.0 * (r + 1)] * 5)


CASES = [(0, 256, 150, 0, 0.6, 1234), (1, 128, 99, 0, 0.42, 77)]


def _system(lat, m, n, pbc, p, seed):
    nb = api.nbonds(lat, m, n, pbc)
    return api.shuffled_ids(nb, seed), int(p * nb)


def _solve_worker(rank, world, port, backend, case, tol, q, inlib=False, per_device=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        lat, m, n, pbc = case[:4]
        order, tb = _system(*case)
        with api.Context(lat, m, n, pbc, device=rank if per_device else 0) as ctx:
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
            assert ctx.label()["nspan"] > 0
            if inlib:  # perc_dslab_solve: the loop inside libperc, own RCCL communicator
                ctx.set_march_mode(PL.MARCH_ALT)
                r = dslab.solve(ctx, tol=tol, itmax=100000)
                r2 = dslab.solve(ctx, tol=tol, itmax=100000)  # communicator reused
                assert [r2[k] for k in ("iter", "gtop", "gbot", "err")] == \
                    [r[k] for k in ("iter", "gtop", "gbot", "err")]
            else:
                r = dslab.conductance(ctx, tol=tol, itmax=100000, check_every=16)
        q.put((rank, r))
    finally:
        dist.destroy_process_group()


def _run(world, backend, case, tol, inlib=False, per_device=False):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.spawn(_solve_worker, args=(world, free_port(), backend, case, tol, q, inlib, per_device),
             nprocs=world, join=True)
    out = {}
    while not q.empty():
        r, res = q.get()
        out[r] = res
    assert sorted(out) == list(range(world))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=["sq256x150", "tri128x99"])
@pytest.mark.parametrize("K", [2, 3])
def test_processes_equal_slabs_in_one_process(case, K):
    lat, m, n, pbc = case[:4]
    order, tb = _system(*case)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        ctx.set_march_mode(PL.MARCH_ALT)  # the slabs run the row-major q-storing march
        ctx.set_slabs(K)
        ref = ctx.conductance(tol=1e-12, itmax=100000)
    out = _run(K, "gloo", case, 1e-12)
    for r in range(K):  # every process reports the same numbers: perc_set_slabs(K)'s
        assert out[r]["iter"] == ref["iter"], (r, out[r], ref)
        assert out[r]["gtop"] == ref["gtop"] and out[r]["gbot"] == ref["gbot"], (r, out[r], ref)


@pytest.mark.gpu
def test_one_process_over_rccl():
    case = CASES[0]
    lat, m, n, pbc = case[:4]
    order, tb = _system(*case)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        ref = ctx.conductance(tol=1e-12, itmax=100000)
    out = _run(1, "nccl", case, 1e-12)[0]
    assert abs(out["iter"] - ref["iter"]) <= 2
    assert abs(out["gtop"] - ref["gtop"]) <= 1e-9 * abs(ref["gtop"])
    assert abs(out["gbot"] - ref["gbot"]) <= 1e-9 * abs(ref["gbot"])


# ------------------------------------------------- the loop inside libperc
def _group(K, case, xport, tol, ordering=None):
    """K labeled contexts on the box's one GPU, one solve split over them by
    perc_dslab_solve_group (one host thread per context)"""
    lat, m, n, pbc = case[:4]
    order, tb = _system(*case)
    ctxs = [api.Context(lat, m, n, pbc) for _ in range(K)]
    try:
        for c in ctxs:
            c.set_march_mode(PL.MARCH_ALT)
            c.occupy(PL.BOND, bond_order=order, nbonds_=tb)
            c.label()
        return api.dslab_solve_group(ctxs, xport=xport, tol=tol, itmax=100000)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=["sq256x150", "tri128x99"])
@pytest.mark.parametrize("K", [2, 3, 4])
def test_group_solve_equals_slabs_in_one_context(case, K):
    """perc_dslab_solve_group with the host transport (K contexts, K host
    threads, one GPU): perc_set_slabs(K)'s numbers bitwise"""
    lat, m, n, pbc = case[:4]
    order, tb = _system(*case)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        ctx.set_march_mode(PL.MARCH_ALT)
        ctx.set_slabs(K)
        ref = ctx.conductance(tol=1e-12, itmax=100000)
    got = _group(K, case, PL.XPORT_HOST, 1e-12)
    assert got["iter"] == ref["iter"] and got["err"] == ref["err"], (got, ref)
    assert got["gtop"] == ref["gtop"] and got["gbot"] == ref["gbot"], (got, ref)


@pytest.mark.gpu
def test_group_solve_over_rccl_one_device():
    """K = 1: the RCCL transport with the exchange forced (ncclCommInitAll on
    the one GPU, one-rank all-gathers and the slab-order combines), the host
    transport with it forced, and the plain K = 1 path (the one-slab kernel
    epilogues, no combine) give the same numbers bitwise -- the combine over
    one partial is the same arithmetic; against the single-context solve
    they differ only in the dot association (the slab kernels' grids)"""
    case = CASES[0]
    lat, m, n, pbc = case[:4]
    order, tb = _system(*case)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.set_march_mode(PL.MARCH_ALT)
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        ref = ctx.conductance(tol=1e-12, itmax=100000)
    key = lambda r: (r["iter"], r["gtop"], r["gbot"], r["err"])  # noqa: E731
    rc = _group(1, case, PL.XPORT_RCCL | PL.XPORT_EXCHANGE, 1e-12)
    rc2 = _group(1, case, PL.XPORT_RCCL | PL.XPORT_EXCHANGE, 1e-12)  # cached communicator
    ho = _group(1, case, PL.XPORT_HOST | PL.XPORT_EXCHANGE, 1e-12)
    solo = _group(1, case, PL.XPORT_RCCL, 1e-12)
    assert key(rc) == key(ho) == key(solo) == key(rc2), (rc, ho, solo)
    assert abs(rc["iter"] - ref["iter"]) <= 2
    assert abs(rc["gtop"] - ref["gtop"]) <= 1e-9 * abs(ref["gtop"])
    assert abs(rc["gbot"] - ref["gbot"]) <= 1e-9 * abs(ref["gbot"])


@pytest.mark.gpu
def test_per_process_solve_world_one():
    """perc_dslab_solve (one process per GPU, its own RCCL communicator from
    rank 0's unique id, the loop inside libperc) at world 1: the group
    solver's numbers bitwise; the second call reuses the communicator"""
    case = CASES[0]
    got = _run(1, "gloo", case, 1e-12, inlib=True)[0]
    want = _group(1, case, PL.XPORT_RCCL, 1e-12)
    assert (got["iter"], got["gtop"], got["gbot"], got["err"]) == \
        (want["iter"], want["gtop"], want["gbot"], want["err"]), (got, want)


def _failure_worker(rank, world, port, case, q):
    """world 1: a rank whose local preparation fails (the literal dot order,
    which a split solve cannot run) must still reach perc_dslab_solve's
    agreement all-reduce and return the error through it -- not before it,
    where peers would wait forever -- and the communicator stays
    usable for the next call"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lat, m, n, pbc = case[:4]
        order, tb = _system(*case)
        with api.Context(lat, m, n, pbc) as ctx:
            ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
            assert ctx.label()["nspan"] > 0
            ctx.set_march_mode(PL.MARCH_ALT)
            ctx.set_dot_order(PL.DOT_LITERAL)
            try:
                dslab.solve(ctx, tol=1e-10, itmax=100000)
                failed = None
            except PL.PercError as e:
                failed = str(e)
            ctx.set_dot_order(PL.DOT_FAST)
            r = dslab.solve(ctx, tol=1e-10, itmax=100000)
        q.put((rank, failed, r))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_per_process_solve_failure_is_agreed():
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.spawn(_failure_worker, args=(1, free_port(), CASES[0], q), nprocs=1, join=True)
    rank, failed, r = q.get()
    assert failed is not None and "literal" in failed, failed
    assert r["iter"] > 0 and r["gtop"] > 0, r


# ------------------------------------------------- several GPUs (skipped on one-GPU boxes)
# The pool's boxes have one GPU: these K = 2 RCCL paths -- the ncclSend /
# ncclRecv halo swap, the all-gather across devices, the top-row hand-off
# (group: hipMemcpyPeer; per process: ncclSend / ncclRecv) -- have not run on
# hardware yet ("Unverified on hardware").
two_gpus = pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                              reason="needs 2 GPUs (RCCL allows one rank per device)")


@pytest.mark.gpu
@two_gpus
def test_group_solve_over_rccl_two_devices():
    """perc_dslab_solve_group over RCCL with slab s on device s (K = 2):
    perc_set_slabs(2)'s numbers in one context, bitwise"""
    case = CASES[0]
    lat, m, n, pbc = case[:4]
    order, tb = _system(*case)
    with api.Context(lat, m, n, pbc) as ctx:
        ctx.occupy(PL.BOND, bond_order=order, nbonds_=tb)
        ctx.label()
        ctx.set_march_mode(PL.MARCH_ALT)
        ctx.set_slabs(2)
        ref = ctx.conductance(tol=1e-12, itmax=100000)
    ctxs = [api.Context(lat, m, n, pbc, device=d) for d in range(2)]
    try:
        for c in ctxs:
            c.set_march_mode(PL.MARCH_ALT)
            c.occupy(PL.BOND, bond_order=order, nbonds_=tb)
            c.label()
        got = api.dslab_solve_group(ctxs, xport=PL.XPORT_RCCL, tol=1e-12, itmax=100000)
    finally:
        for c in ctxs:
            c.close()
    assert (got["iter"], got["err"], got["gtop"], got["gbot"]) == \
        (ref["iter"], ref["err"], ref["gtop"], ref["gbot"]), (got, ref)


@pytest.mark.gpu
@two_gpus
def test_per_process_solve_two_devices():
    """perc_dslab_solve, one process per GPU (K = 2, RCCL from rank 0's
    unique id): both ranks report the group solver's numbers bitwise"""
    case = CASES[0]
    out = _run(2, "gloo", case, 1e-12, inlib=True, per_device=True)
    lat, m, n, pbc = case[:4]
    order, tb = _system(*case)
    ctxs = [api.Context(lat, m, n, pbc, device=d) for d in range(2)]
    try:
        for c in ctxs:
            c.set_march_mode(PL.MARCH_ALT)
            c.occupy(PL.BOND, bond_order=order, nbonds_=tb)
            c.label()
        want = api.dslab_solve_group(ctxs, xport=PL.XPORT_RCCL, tol=1e-12, itmax=100000)
    finally:
        for c in ctxs:
            c.close()
    for r in range(2):
        assert (out[r]["iter"], out[r]["gtop"], out[r]["gbot"]) == \
            (want["iter"], want["gtop"], want["gbot"]), (r, out[r], want)
