"""Ensemble sharding of independent realisations over ranks (one process
per GPU) and the one collective of the path: the all-reduce of the
ensemble statistics (Square/bond_cond.f:62-70 seeds each
trial ii from the master seed, trials are independent).

  rank r of W handles ii = k*W + r (k = 0, 1, ...), seed tseed(ii);
  stats = [count, sum G, sum G^2, count spanning, sum iter] (+ per grid
  point for bond_cond sweeps), summed over ranks; elapsed = max over ranks.

With backend "nccl" the all-reduce is RCCL over xGMI; the same code runs
with "gloo" on CPU (tests/test_ensemble_gloo.py).
"""
import numpy as np

NSTAT = 5  # count, sum G, sum G^2, spanning, sum iter


def trial_indices(nreal, world, rank, nseeds=1000):
    """0-based trial ids of this rank's nreal realisations: trial ii (0-based)
    runs on rank ii mod world, as perc_ensemble_trials stripes devices.  The
    reference never reuses a seed (tseed(1..1000), bond_cond.f:67), so an
    ensemble larger than the seeds generated is an error, not a wrap."""
    if nreal * world > nseeds:
        raise ValueError("ensemble of %d x %d realisations exceeds the %d trial seeds; "
                         "generate more seeds (perc_trial_seeds with k >= %d)"
                         % (nreal, world, nseeds, nreal * world))
    return [k * world + rank for k in range(nreal)]


def local_stats(results):
    """Stats vector of this rank's realisations (dicts with gtop, nspan,
    iter)."""
    g = np.array([r["gtop"] for r in results], dtype=np.float64)
    return np.array([len(results), g.sum(), (g * g).sum(),
                     sum(1 for r in results if r["nspan"] > 0),
                     sum(r["iter"] for r in results)], dtype=np.float64)


def grid_stats(rows_per_trial, npts):
    """bond_cond sweeps: per grid point [count, sum G, sum G^2, spanning,
    sum iter] over this rank's trials, shape (npts, NSTAT)."""
    acc = np.zeros((npts, NSTAT))
    for rows in rows_per_trial:
        for j, r in enumerate(rows[:npts]):
            acc[j] += (1, r["gtop"], r["gtop"] ** 2, 1 if r["spanning"] else 0, r["iter"])
    return acc


def allreduce(stats, elapsed, device="cpu"):
    """Sum `stats` and take the max of `elapsed` over all ranks (a no-op
    without an initialised process group).  Returns (stats, elapsed)."""
    import torch
    import torch.distributed as dist
    s = torch.as_tensor(np.asarray(stats, dtype=np.float64), device=device).clone()
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return s.cpu().numpy(), float(t.item())


def summary(stats):
    """Mean/variance of G, spanning fraction and mean iterations from a
    (reduced) stats vector."""
    n = max(stats[0], 1.0)
    mean = stats[1] / n
    return dict(count=int(stats[0]), gtop_mean=mean,
                gtop_var=max(stats[2] / n - mean * mean, 0.0),
                spanning_fraction=stats[3] / n, iter_mean=stats[4] / n)
