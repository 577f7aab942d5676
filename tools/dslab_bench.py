#!/usr/bin/env python3
"""Per-iteration cost of the split solve's machinery at K = 1 (one GPU):
the single-context solve with the slab kernels' march (MARCH_ALT, q stored)
against perc_dslab_solve_group -- plain K = 1 (one-slab epilogues, no
exchange), and with PERC_XPORT_EXCHANGE forcing the slab-order combines and
one-rank collectives over RCCL and through the host -- and, with --torch,
percolation_amd/dslab.py's Python loop over a torch.distributed "nccl" group
of one (in a child process of its own: torch's bundled RCCL and libperc's
are separate copies).  Fixed iteration counts (tol 0): ms per iteration =
the slope between solves of iters / 2 and iters iterations, best of --reps
(set-up, the cached communicator and the currents cancel).

  python tools/dslab_bench.py --L 4096 --iters 2000 [--torch]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--torch-leg", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    from percolation_amd import _lib as PL
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    tb = int(args.p * nb)
    seed = int(api.trial_seeds(58302, 1)[0])
    out = dict(L=L_, p=args.p, iterations=args.iters, reps=args.reps)

    def ctx_new():
        c = api.Context(0, L_, L_, 0)
        c.set_march_mode(PL.MARCH_ALT)
        c.occupy_random(PL.BOND, 0, tb, seed)
        c.label()
        return c

    def slope(fn):
        fn(50)  # warm (and the communicator)
        best = {}
        for _ in range(args.reps):
            for n in (args.iters // 2, args.iters):
                t = time.perf_counter()
                it = fn(n - 1)
                dt = time.perf_counter() - t
                if n not in best or dt < best[n][0]:
                    best[n] = (dt, it)
        (t1, i1), (t2, i2) = best[args.iters // 2], best[args.iters]
        return round((t2 - t1) * 1e3 / (i2 - i1), 5)

    if args.torch_leg:
        import torch
        import torch.distributed as dist
        from percolation_amd import dslab
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        import faulthandler
        faulthandler.enable()  # (an abort names the Python line it came from)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        c = ctx_new()
        print("torch leg: context ready", file=sys.stderr, flush=True)
        ms = slope(lambda n: dslab.conductance(c, tol=0.0, itmax=n)["iter"])
        print("torch leg: timed", file=sys.stderr, flush=True)
        c.close()
        print("torch leg: context closed", file=sys.stderr, flush=True)
        dist.destroy_process_group()
        print("torch leg: group destroyed", file=sys.stderr, flush=True)
        print(json.dumps({"python_dslab_nccl_ms_per_it": ms}), flush=True)
        return  # (normal teardown: one HIP runtime per process, _lib._one_runtime)
    # every leg measured once per round, the legs interleaved round after
    # round (clock and power state drift between legs otherwise), best of rounds
    legs = [("single_context", None), ("group_k1", PL.XPORT_RCCL),
            ("group_rccl_exchange", PL.XPORT_RCCL | PL.XPORT_EXCHANGE),
            ("group_host_exchange", PL.XPORT_HOST | PL.XPORT_EXCHANGE)]
    ctxs = {name: ctx_new() for name, _ in legs}

    def run(name, xp, n):
        c = ctxs[name]
        if xp is None:
            return c.conductance(tol=0.0, itmax=n)["iter"]
        return api.dslab_solve_group([c], xport=xp, tol=0.0, itmax=n)["iter"]
    for name, xp in legs:
        run(name, xp, 50)  # warm (and the communicator)
    best = {}
    for _ in range(args.reps):
        for name, xp in legs:
            for n in (args.iters // 2, args.iters):
                t = time.perf_counter()
                it = run(name, xp, n - 1)
                dt = time.perf_counter() - t
                if (name, n) not in best or dt < best[(name, n)][0]:
                    best[(name, n)] = (dt, it)
    for name, _ in legs:
        (t1, i1), (t2, i2) = best[(name, args.iters // 2)], best[(name, args.iters)]
        out[name + "_ms_per_it"] = round((t2 - t1) * 1e3 / (i2 - i1), 5)
    for c in ctxs.values():
        c.close()
    if args.torch:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--L", str(L_), "--p", str(args.p),
                            "--iters", str(args.iters), "--reps", str(args.reps), "--torch-leg"],
                           capture_output=True, text=True, timeout=600)
        sys.stderr.write(r.stderr[-2000:])
        if r.returncode == 0:
            out.update(json.loads(r.stdout.strip().splitlines()[-1]))
        else:
            out["python_dslab_nccl_error"] = f"rc={r.returncode}"
    for k in [k[:-len("_ms_per_it")] for k in out if k.endswith("_ms_per_it")]:
        if k != "single_context":
            out[k + "_overhead_us"] = round((out[k + "_ms_per_it"] - out["single_context_ms_per_it"]) * 1e3, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
