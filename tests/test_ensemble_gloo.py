"""Multi-rank path of the ensemble (percolation_amd/ensemble.py, used by
bench.py) with world size 2 over gloo on CPU: the trial shards are
disjoint and cover the ensemble, and the all-reduced statistics equal the
single-process statistics of all realisations.  The realisations here are
produced by the host label replay (no GPU): trial ii -> tseed(ii) ->
reference shuffle -> spanning label -> a deterministic stand-in "G"."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from percolation_amd import _lib as PL
from percolation_amd import api, ensemble

L_, P_, NREAL = 24, 0.55, 5


def realisation(ii, seeds):
    nb = api.nbonds(0, L_, L_, 0)
    order = api.shuffled_ids(nb, int(seeds[ii]))
    r = api.replay_labels(0, L_, L_, 0, PL.BOND, bond_order=order, nbond=int(P_ * nb))
    span = r["perccln"] > 0
    g = float(r["csize"][r["perccln"]]) / nb if span else 0.0
    return dict(gtop=g, nspan=1 if span else 0, iter=int(r["maxcs"]))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seeds = api.trial_seeds(58302, 1000)
        ids = ensemble.trial_indices(NREAL, world, rank)
        res = [realisation(ii, seeds) for ii in ids]
        stats, el = ensemble.allreduce(ensemble.local_stats(res), elapsed=1.0 + rank)
        q.put((rank, ids, stats.tolist(), el))
    finally:
        dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shards_disjoint_and_cover():
    w = 4
    ids = [ensemble.trial_indices(10, w, r) for r in range(w)]
    flat = sorted(i for s in ids for i in s)
    assert flat == list(range(40))


def test_world2_gloo_stats_equal_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    seeds = api.trial_seeds(58302, 1000)
    all_ids = sorted(i for _, ids, _, _ in out for i in ids)
    assert all_ids == sorted(set(all_ids)) and len(all_ids) == world * NREAL
    ref = ensemble.local_stats([realisation(ii, seeds) for ii in all_ids])
    for _, _, stats, el in out:
        assert np.allclose(stats, ref, rtol=1e-14, atol=0)
        assert el == 2.0  # max over ranks
    s = ensemble.summary(np.array(out[0][2]))
    assert s["count"] == world * NREAL and 0 <= s["spanning_fraction"] <= 1


def test_grid_stats_shape():
    rows = [[dict(gtop=0.1, spanning=True, iter=3), dict(gtop=0.0, spanning=False, iter=0)]]
    acc = ensemble.grid_stats(rows, 3)
    assert acc.shape == (3, ensemble.NSTAT) and acc[0, 0] == 1 and acc[2, 0] == 0
