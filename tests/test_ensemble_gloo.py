"""Multi-rank path of the ensemble (percolation_amd/ensemble.py, used by
bench.py) with world size 2 over gloo on CPU: the trial shards are
disjoint and cover the ensemble, and the all-reduced statistics equal the
single-process statistics of all realisations.  With no GPU here, each
rank's realisations are the oracle's (tests only: oracle/perc_oracle.c):
trial ii -> tseed(ii) -> reference shuffle -> labels -> the spanning
cluster's conductance by the literal linbcg (Square/bondc.f:189-595).
Also the device striping of perc_ensemble (include/perc.h) for 2-8 virtual
devices: ii -> device (ii-1) mod ndev, every trial exactly once, rows
gathered in ii order."""
import json
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from percolation_amd import api, ensemble

L_, P_, NREAL = 24, 0.55, 5


def realisation(ii, seeds):
    """oracle bondc realisation (labels, spanning, Kirchhoff system, linbcg,
    terminal currents) for trial ii's seed; G = 0 when nothing spans."""
    r = O.bondc(0, L_, L_, 0, P_, int(seeds[ii]))
    span = r["perccln"] > 0
    return dict(gtop=r["gtop"] if span else 0.0, nspan=1 if span else 0,
                iter=r["iter"] if span else 0)


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


def test_trial_indices_never_wrap():
    with pytest.raises(ValueError):
        ensemble.trial_indices(300, 4, 0, nseeds=1000)


@pytest.mark.parametrize("ndev", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("ntrials", [1, 7, 512])
def test_device_striping_and_gather_order(ndev, ntrials):
    """perc_ensemble_trials (C) == ensemble.trial_indices (bench ranks), every
    trial on exactly one device, and gathering each device's rows into slot
    ii-1 reproduces the serial ii order."""
    owner = np.full(ntrials + 1, -1)
    slots = [None] * ntrials
    for d in range(ndev):
        ii = api.ensemble_trials(ntrials, ndev, d)
        assert list(ii) == list(range(d + 1, ntrials + 1, ndev))
        k = len(ii)
        if ntrials >= ndev * k:  # whole rounds: the ranks' 0-based ids
            assert [i - 1 for i in ii] == ensemble.trial_indices(k, ndev, d, nseeds=ntrials)
        for i in ii:
            assert owner[i] == -1
            owner[i] = d
            slots[i - 1] = ("row", i)  # what device d writes for trial i
    assert (owner[1:] >= 0).all()
    assert slots == [("row", i) for i in range(1, ntrials + 1)]


def test_seeded_shuffle_equals_global_stream():
    """the per-thread shuffle of perc_ensemble equals srand + the REAL*4
    Fisher-Yates on the global stream (bondc.f:162-174)"""
    for n, seed in [(40, 4562929), (2000, 123), (5, 0)]:
        a = np.zeros(n + 1, np.int32)
        from percolation_amd import _lib as PL
        PL.lib().perc_shuffle_seeded(seed, n, a)
        b = api.shuffled_ids(n, seed)
        assert np.array_equal(a[:n], b[:n])


def test_ensemble_without_device_fails_loudly():
    import ctypes as C
    import torch
    from percolation_amd import _lib as PL
    if torch.cuda.is_available():
        pytest.skip("device present")
    h = C.c_void_p()
    assert PL.lib().perc_ensemble_create(2, None, 0, 16, 16, 0, C.byref(h)) == -8


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


def _bench(*args, timeout=120):
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(repo, "bench.py")] + list(args),
                          capture_output=True, text=True, timeout=timeout, env=env)


def test_bench_gpus_n_launches_n_ranks():
    """bench.py --gpus N without torch.distributed.run starts N rank processes
    itself (bench.launch_ranks); here the ranks run the gloo stub: one group
    of world size 2, one all-reduce, rank 0's JSON line relayed."""
    r = _bench("--gpus", "2", "--launch-stub")
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out == {"n_gpus": 2, "allreduce_sum": 3.0, "local_ranks": 2}


def test_bench_gpus_n_more_than_visible_fails_loudly():
    """--gpus N with fewer visible GPUs (none here) is an error, not a
    one-GPU run reported as N"""
    r = _bench("--gpus", "2")
    assert r.returncode != 0
    assert "visible GPU" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
