#!/usr/bin/env python3
"""Benchmark: conductance solves/s + CG SpMV GB/s on the BASELINE.json metric
workload (square L=4096 bond percolation at p=0.60, bondc semantics).

One "step" = one realisation through the whole hot path: occupancy drawn
on the GPU (perc_occupy_random; or from a device-resident order drawn on
the host, --occupancy uniform), GPU labeling + spanning, Kirchhoff
assembly, fused Jacobi-PCG to tol 1e-8 (linbcg stopping rule, itmax 1e6),
terminal currents.  Realisations shard across ranks (ii = step*world+rank,
seeds tseed(ii) from master 58302, bond_cond.f:65-70); the only collective
is the RCCL all-reduce of the ensemble statistics.  Weak scaling.

  python bench.py [--gpus N --steps K --warmup W --L 4096 --p 0.6]
  torchrun --nproc-per-node N bench.py --gpus N ...

`--gpus N` without a launcher starts the N rank processes itself
(launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as
torch.distributed.run sets them, before any GPU call in the parent); each
rank then runs its share of the realisations on its GPU.
"""
import argparse
import json
import os
import re
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmv_bytes(N, nnz, fmt):
    """Algorithmic bytes of one SpMV (k_cg_spmv / k_spmv), p read once and q
    written once (the q.p dot adds no traffic).
    csr: SURVEY.md §8(d) B = 8(N+nnz) + 4 nnz + 4(N+1) + 16N -- diagonal and
         off-diagonal values, column indices, row pointers, p, q;
    stencil: a 2-byte code per row + p + q = 18N (columns, values and the
         diagonal are rebuilt from the code and the row-form table)."""
    if fmt == "csr":
        return 8 * (N + nnz) + 4 * nnz + 4 * (N + 1) + 16 * N
    return 18 * N


def x_bytes(N, m, full):
    """x += ak p: read + write of x on every row (full voltages), or on the
    two interior rows next to the electrodes only (perc_set_full_voltages
    off: the currents read no other voltage, bondc.f:554-592)."""
    return 16 * N if full else 16 * 2 * m


def ps_bytes(N, m, full, qfree=False):
    """Fused P(k)+S(k) (p update + SpMV + q.p; march or LDS tiles): reads
    p(k-1), r, code; writes p(k) and, unless the B kernel rebuilds q
    (q-free march), q -- 34N (26N q-free), plus x (halo re-reads are not
    algorithmic; they show in the PMC traffic)."""
    return (26 if qfree else 34) * N + x_bytes(N, m, full)


def resid_bytes(N, fmt):
    """B: reads r, q and d (csr: 8 B diag, stencil: 2 B code); writes r.  The
    q-free march B reads p(k) instead of q: the same 26N."""
    return 32 * N if fmt == "csr" else 26 * N


def xp_bytes(N, fmt, m, full):
    """k_cg_p: reads p, r and d (csr: 8 B, stencil: 2 B); writes p; plus x."""
    return (32 * N if fmt == "csr" else 26 * N) + x_bytes(N, m, full)


KERNELS = {"pm": "march kernel (fused p = bk p + r/d, x += ak p, q = A p, q.p)",
           "ps": "k_cg_ps (fused p = bk p + r/d, x += ak p, q = A p, q.p; LDS tiles)",
           "spmv": "k_cg_spmv (SpMV q = A p + q.p dot)",
           "resid": "k_cg_b (r -= ak q, z = r/d, z.r and r.r dots)",
           "xp": "k_cg_p (x += ak p, p = bk p + r/d)"}


def cpu_baseline(L_, p, order, gpu_iters, cpu_iters, tol=1e-8):
    """The oracle (oracle/perc_oracle.c, a serial C restatement of the
    reference path, bit-exact against it) on one host core, on a bounded
    sample of the same workload: union-find labeling + assembly + `cpu_iters`
    linbcg iterations + currents of the first timed L x L realisation (same
    occupation order); the solve is extrapolated to the GPU's iteration
    count for that realisation.  cpu_iters <= 0: the whole solve to `tol`,
    measured end to end (no extrapolation)."""
    import ctypes as C

    import oracle_lib as O
    Or = O.lib()
    lat, m, n = 0, L_, L_
    t, N = m * n, m * n - 2 * m
    b1, b2 = O.bond_list(lat, m, n, 0)
    nb = len(b1)
    tb = len(order)
    o1, o2 = O.i32(nb + 1), O.i32(nb + 1)
    ids = order[order > 0] - 1
    o1[:len(ids)], o2[:len(ids)] = b1[ids], b2[ids]
    label, cs = O.i32(nb), O.i32(nb + 2)
    mx, ms = C.c_int(), C.c_int()
    t0 = time.perf_counter()
    cln = Or.or_label_bonds_replay(lat, m, n, 0, nb, b1, b2, o1, o2, tb, label, cs, C.byref(mx),
                                   C.byref(ms))
    perc = Or.or_span_bonds(m, n, nb, b1, b2, label, cs, cln)
    t1 = time.perf_counter()
    del o1, o2
    gval = O.f64(nb)
    Or.or_bond_values(0, nb, b1, b2, label, O.i32(1), perc, 1.0, 1e-12, gval)
    nmax = N + 1 + 2 * nb + 8
    sa, ija = O.f64(nmax), O.i32(nmax)
    itemp, diag = O.f64(N), O.f64(t)
    Or.or_assemble(lat, m, n, 0, nb, b1, b2, gval, 1.0, 1e-16, 0, nmax, sa, ija, itemp, diag)
    t2 = time.perf_counter()
    vint = O.f64(N)
    it, err = C.c_int(), C.c_double()
    if cpu_iters > 0:
        Or.or_linbcg(sa, ija, N, itemp, vint, 2, -1.0, cpu_iters - 1, C.byref(it), C.byref(err),
                     None)
    else:
        Or.or_linbcg(sa, ija, N, itemp, vint, 2, tol, 10 ** 7, C.byref(it), C.byref(err), None)
        gpu_iters = it.value
    t3 = time.perf_counter()
    gt, gb = C.c_double(), C.c_double()
    Or.or_currents(lat, m, n, 0, nb, b1, b2, gval, diag, vint, 1.0, 1e-10, 0, C.byref(gt),
                   C.byref(gb))
    t4 = time.perf_counter()
    per_iter = (t3 - t2) / it.value
    total = (t1 - t0) + (t2 - t1) + per_iter * gpu_iters + (t4 - t3)
    how = ("%d linbcg iterations to tol %g (%.3fs/it), measured whole" % (it.value, tol, per_iter)
           if cpu_iters <= 0 else "%d linbcg iterations (%.3fs/it, extrapolated to the GPU's %d)"
           % (it.value, per_iter, gpu_iters))
    return dict(value=1.0 / total, unit="solves/s", cores=1, kind="port",
                sample=("oracle C restatement (perc_oracle.c) on 1 core: union-find labeling "
                        "%.2fs + assembly %.2fs + %s + currents %.2fs, one L=%d p=%.2f realisation"
                        % (t1 - t0, t2 - t1, how, t4 - t3, L_, p)),
                sample_seconds=round(t4 - t0, 2), s_per_solve=round(total, 2),
                measured_seconds=round(t4 - t0, 2), iterations=it.value,
                extrapolated=cpu_iters > 0, t_label=t1 - t0, t_assemble=t2 - t1,
                s_per_iter=per_iter, t_currents=t4 - t3,
                # the sample's currents: only after a whole solve is this the
                # realisation's conductance (a bounded sample stops at
                # cpu_iters iterations, far from converged)
                **({"gtop_converged": gt.value} if cpu_iters <= 0
                   else {"gtop_unconverged_after_sample": gt.value}))


def cpu_anchor_start(L_, p, seed, iters, occupancy):
    """Start one 1-core oracle process (cpu_worker) in the background, so the
    CPU anchor runs on its own host core while the GPU realisations run"""
    import subprocess
    lat_nb = (2 * L_ * L_ - 2 * L_)
    env = dict(os.environ, PERC_BENCH_OCCUPANCY=occupancy, OMP_NUM_THREADS="1")
    return subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-iters", str(iters),
                             "--cpu-worker", str(L_), str(p), str(int(seed)), "0", str(lat_nb),
                             str(int(p * lat_nb))],
                            stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, env=env)


def cpu_anchor_finish(proc, gpu_iters=None):
    out, _ = proc.communicate()
    if proc.returncode != 0 or not out.strip():
        return {"value": None, "error": "cpu anchor process failed (rc %s)" % proc.returncode}
    r = json.loads(out.strip().splitlines()[-1])
    if r.get("extrapolated") and gpu_iters:  # the sample's rate, extrapolated to the GPU's count
        total = r["t_label"] + r["t_assemble"] + r["s_per_iter"] * gpu_iters + r["t_currents"]
        r["value"], r["s_per_solve"] = 1.0 / total, round(total, 2)
        r["sample"] = r["sample"].replace("extrapolated to the GPU's 0", "extrapolated to the GPU's %d"
                                          % gpu_iters)
    return r


def cpu_worker(spec, cpu_iters):
    """One process of the all-cores CPU ensemble baseline: the 1-core
    sample of cpu_baseline on its own realisation (spec = L, p, seed,
    iters, nb, tb; the order drawn as main() draws it)."""
    L_, p, seed, iters, nb, tb = (int(spec[0]), float(spec[1]), int(spec[2]), int(spec[3]),
                                  int(spec[4]), int(spec[5]))
    if os.environ.get("PERC_BENCH_OCCUPANCY") == "device":  # the keys' order (host, libperc)
        from percolation_amd import api
        order = np.ascontiguousarray(api.random_order(nb, tb, seed), dtype=np.int32)
    else:
        order = (np.random.default_rng(seed).permutation(nb)[:tb] + 1).astype(np.int32)
    print(json.dumps(cpu_baseline(L_, p, order, iters, cpu_iters)), flush=True)


def cpu_ensemble(L_, p, seeds, iters, nb, tb, cpu_iters, cores, occupancy="uniform"):
    """ensemble throughput of the CPU path with all host
    cores, one independent realisation per core (child processes running
    cpu_worker concurrently, so memory-bandwidth contention is included)."""
    import subprocess
    t0 = time.perf_counter()
    env = dict(os.environ, PERC_BENCH_OCCUPANCY=occupancy)
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-iters",
                               str(cpu_iters), "--cpu-worker", str(L_), str(p), str(int(sd)),
                               str(iters), str(nb), str(tb)],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, env=env)
             for sd in seeds[:cores]]
    res = []
    for pr in procs:
        out, _ = pr.communicate()
        if pr.returncode == 0 and out.strip():
            res.append(json.loads(out.strip().splitlines()[-1]))
    if not res:
        return {"value": None, "error": "no worker finished"}
    per = [r["s_per_solve"] for r in res]
    return {"value": round(sum(1.0 / x for x in per), 8), "unit": "solves/s", "cores": len(res),
            "kind": "port",
            "sample": "%d concurrent processes, each the 1-core sample of cpu_baseline on its own "
                      "realisation (labeling + assembly + %d linbcg iterations + currents, solve "
                      "extrapolated to %d iterations, the GPU mean); value = sum of per-process "
                      "rates" % (len(res), cpu_iters, iters),
            "s_per_solve_mean": round(float(np.mean(per)), 2),
            "wall_seconds": round(time.perf_counter() - t0, 2)}


def labeling_probe(ctx, P, L_, nb, tb, seeds, kind="bond", ts=0):
    """Occupancy draw, labeling + spanning test and Kirchhoff assembly of
    the timed realisations again, phase by phase after a synchronize (best
    of the seeds), outside the timed region.  Algorithmic bytes
    (Square/bondc.f:194-393 labels, :482-532 assembly; sitebond.f:187-458;
    t = L^2 sites, N = interior rows, F = the occupancy flag bytes: nb bond
    flags, t site flags, nb + t mixed): occupy writes the u8 flags (F);
    labeling reads them and writes the int32 parent and u8 member arrays
    (F + 5t); assembly reads flags, parents and members (F + 5t) and writes
    the u16 row codes and the f64 right-hand side (10N) -- only for the
    realisations that span.  The roofline is 8 TB/s."""
    import torch
    t = L_ * L_
    N = t - 2 * L_
    lk = {"bond": P._lib.BOND, "site": P._lib.SITE, "sitebond": P._lib.SITEBOND}[kind]
    rule = {"bond": P._lib.RULE_BOND, "site": P._lib.RULE_SITE, "sitebond": P._lib.RULE_MIXED}[kind]
    F = {"bond": nb, "site": t, "sitebond": nb + t}[kind]
    ctx.set_matrix_format(P.FMT_AUTO)  # (the kernel probe left the last format set)
    best, best_asm = None, None
    for sd in seeds:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.occupy_random(lk, ts if kind != "bond" else 0, tb if kind != "site" else 0, sd)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        li = ctx.label()
        t2 = time.perf_counter()
        row = ((t1 - t0) * 1e3, (t2 - t1) * 1e3)
        best = row if best is None else tuple(min(a, b) for a, b in zip(best, row))
        if li["nspan"]:
            c = ctx.conductance(rule, tol=1e-8, itmax=1)
            best_asm = c["t_assemble_ms"] if best_asm is None else min(best_asm, c["t_assemble_ms"])
    if best is None:
        return None
    phases = {"occupy": (best[0], F), "label": (best[1], F + 5 * t)}
    if best_asm is not None:
        phases["assemble"] = (best_asm, F + 5 * t + 10 * N)
    out = {k: {"ms": round(ms, 4), "bytes": b, "gbs": round(b / (ms * 1e-3) / 1e9, 1),
               "frac": round(b / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
           for k, (ms, b) in phases.items()}
    tot = sum(v[0] for v in phases.values())
    out["total_ms"] = round(tot, 4)
    out["note"] = ("per realisation, best of %d, wall time after a synchronize (label includes "
                   "the spanning test's host read-back)" % len(seeds))
    return out


def kernel_label(key, minfo):
    """Name + role of a CG kernel, for the march variant that ran."""
    if key == "pm" and minfo.get("kernel") == "wave":
        return "k_cg_march (per-wave register march %d cols x %d rows%s%s%s): fused p = bk p + r/d, " \
            "q = A p, q.p%s" % (
                minfo["strip_cols"], minfo["band_rows"], ", alternating" if minfo["alt"] else "",
                ", strip-major" if minfo.get("strips") else "",
                ", nibble row codes" if minfo.get("nibble") else "",
                "" if minfo["qfree"] else ", q stored")
    if key == "res":
        return ("k_cg_res (resident persistent solve, %d-row bands: p in LDS, r/q in registers, "
                "2 grid-wide reductions per iteration; bytes = the streaming-equivalent 52 B/row "
                "+ x, not HBM traffic)"
                % minfo["band_rows"])
    if key == "resid" and minfo.get("qfree"):
        return "k_cg_march B (march: q = A p(k) rebuilt, r -= ak q, z = r/d, z.r and r.r dots)"
    return KERNELS[key]


# rocprof kernel names of the CG kernels, per operator format
ROCPROF_NAMES = {("res", "stencil"): ("k_cg_res",),  # default kernel of each role first
                 ("res", "stencil_tiled"): ("k_cg_res",),
                 ("pm", "stencil"): ("k_cg_march<1", "k_cg_march<0"),
                 ("ps", "stencil_tiled"): ("k_cg_ps<4>", "k_cg_ps<6>"),
                 ("resid", "stencil_tiled"): ("k_cg_b<true>",),
                 ("spmv", "stencil_split"): ("k_cg_spmv<4>", "k_cg_spmv<6>"),
                 ("resid", "stencil_split"): ("k_cg_b<true>",),
                 ("resid", "stencil"): ("k_cg_march<2", "k_cg_b<true>"),
                 ("xp", "stencil_split"): ("k_cg_p<true>",),
                 ("spmv", "stencil"): ("k_cg_spmv<4>", "k_cg_spmv<6>"),
                 ("spmv", "csr"): ("k_cg_spmv<0>",),
                 ("resid", "csr"): ("k_cg_b<false>",),
                 ("xp", "stencil"): ("k_cg_p<true>",), ("xp", "csr"): ("k_cg_p<false>",)}


def base_name(k):
    """'k_cg_ps<4, false, 1, 1024, 32>' -> 'k_cg_ps<4' (first template argument)"""
    return k.split(",")[0].rstrip(">")


def rocprof_base(key, fmt, minfo):
    """base name (kernel + first template argument, as base_name gives it) of
    the CG kernel of role `key` that the solve ran"""
    if fmt == "stencil" and minfo.get("kernel") == "wave" and key in ("pm", "resid"):
        k = "k_cg_march"
        if key == "pm":
            return "%s<%d" % (k, 1 if minfo.get("qfree") else 0)
        return "%s<2" % k if minfo.get("qfree") else "k_cg_b<true"
    names = ROCPROF_NAMES.get((key, fmt), ())
    return base_name(names[0]) if names else None


def rocprof_avg(base, L_):
    """average duration (ms) of kernel `base` in the newest committed
    rocprofv3 --kernel-trace --stats summary of this lattice size
    (profiles/*_rocprof_stats_L<L>.csv) and its path: the cross-check of the
    live event timing, whose brackets include the dispatch gap before each
    launch.  (None, None) if absent."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_rocprof_stats_L%d.csv" % L_)),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))],
                   reverse=True)
    for f in files if base else ():
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Name") or ""
                i = name.find(base)
                if i >= 0 and name[i + len(base):i + len(base) + 1] in (",", ">"):
                    return float(r["AverageNs"]) / 1e6, os.path.relpath(f, REPO)
    return None, None


# reconcile summaries before r2_17 name kernels without template arguments;
# the kernels they measured
OLD_RECONCILE = {"k_cg_march": "k_cg_march<0", "k_cg_b": "k_cg_b<true"}


def pmc_traffic(base, L_, kind="bond"):
    """HBM bytes per launch of a CG kernel from the committed rocprofv3 PMC
    summaries.  Preferred: profiles/*_pmc_reconcile_L<L>.csv
    (tools/pmc_r2.sh + tools/pmc_reconcile.py): one fixed dispatch set of
    work launches in every pass, read bytes from the 32/64/128-B EA read
    request counters (exact; gfx950's FETCH_SIZE tallies 128-B requests at
    64 B), write bytes from WRITE_SIZE.  Else the older per-counter
    summaries (*_pmc_{fetch,write}_L<L>.csv, FETCH_SIZE doubled).  None if
    absent."""
    import csv
    import glob

    def newest_first(pattern):
        # r<round>_<n> prefixes compared as numbers (file times are not kept
        # by every copy of the tree)
        files = glob.glob(os.path.join(REPO, "profiles", pattern))
        return sorted(files, key=lambda f: [int(t) if t.isdigit() else t
                                            for t in re.split(r"(\d+)", os.path.basename(f))],
                      reverse=True)

    # a mixed occupation's matrix (the config-5 companion) cites its own
    # reconciliation (*_pmc_reconcile_L<L>_mixed.csv) where there is one
    pats = (["*_pmc_reconcile_L%d_mixed.csv" % L_] if kind == "sitebond" else []) + \
        ["*_pmc_reconcile_L%d.csv" % L_]
    for f in [f for pat in pats for f in newest_first(pat)]:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if OLD_RECONCILE.get(r["kernel"], r["kernel"]) == base and r["read_bytes"] \
                        and r["write_bytes"]:
                    return float(r["read_bytes"]) + float(r["write_bytes"]), [os.path.relpath(f, REPO)]
    tot, src = 0.0, []
    for kind, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        got = None
        for f in newest_first("*_pmc_%s_L%d.csv" % (kind, L_)):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if base_name(r["kernel"]) == base and r["counter"] == ctr:
                        got = float(r["bytes_per_dispatch"])
            if got is not None:
                src.append(os.path.relpath(f, REPO))
                break
        if got is None:
            return None, None
        tot += got
    return tot, src


def launch_ranks(n, argv, stub=False):
    """`bench.py --gpus N` without a launcher: start N rank processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run
    sets them) before anything here touches the GPU, wait for them and return
    the first non-zero exit status.  The ranks inherit stdout, so rank 0's
    JSON line is the only line printed.  If one rank fails the others are
    ended (a rank left waiting in a collective would never return)."""
    import signal
    import socket
    import subprocess
    if not stub:
        import torch  # device_count() does not initialise the GPU
        ndev = torch.cuda.device_count()
        if ndev < n:
            log("bench.py --gpus %d: only %d visible GPU(s)" % (n, ndev))
            return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for pr in list(live):
            code = pr.poll()
            if code is None:
                continue
            live.remove(pr)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log("bench.py: rank %d exited with %d; ending the other ranks"
                    % (procs.index(pr), code))
                for o in live:
                    o.send_signal(signal.SIGTERM)
                deadline = time.time() + 20
                for o in live:
                    try:
                        o.wait(max(deadline - time.time(), 0.1))
                    except subprocess.TimeoutExpired:
                        o.kill()
        time.sleep(0.2)
    return rc


def launch_stub():
    """--launch-stub: what a rank of launch_ranks() runs in the CPU test --
    a gloo group of WORLD_SIZE ranks and one all-reduce, rank 0 printing the
    JSON line (n_gpus = the world size the launcher set)."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "allreduce_sum": float(t.item()),
                          "local_ranks": int(os.environ["LOCAL_WORLD_SIZE"])}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.60)
    ap.add_argument("--master", type=int, default=58302)
    ap.add_argument("--tol", type=float, default=1e-8)
    ap.add_argument("--itmax", type=int, default=10 ** 6)
    ap.add_argument("--cpu-iters", type=int, default=500,
                    help="linbcg iterations of the 1-core CPU sample at L (extrapolated to the "
                         "GPU's count); the whole L=1024 anchor solve runs beside it")
    ap.add_argument("--cpu-ensemble-iters", type=int, default=20,
                    help="linbcg iterations of each all-cores ensemble process")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--occupancy", choices=("device", "uniform", "reference"), default="device",
                    help="device: drawn on the GPU inside each realisation (perc_occupy_random, "
                         "counter-based keys from tseed(ii)); uniform: numpy PCG64 permutation "
                         "drawn on the host before the timed region; reference: the reference's "
                         "REAL*4 shuffle (biased above 2^22 bonds, H10)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the RCCL process group even at world size 1 (checks the "
                         "multi-GPU path on one GPU)")
    ap.add_argument("--lattice", choices=("square", "tri"), default="square")
    ap.add_argument("--kind", choices=("bond", "site", "sitebond"), default="bond",
                    help="site / sitebond use the ConductCalc.m site / mixed rules")
    ap.add_argument("--ps", type=float, default=0.593, help="site fraction for --kind sitebond")
    ap.add_argument("--full-voltages", action="store_true",
                    help="update x on every row every iteration (perc_set_full_voltages)")
    ap.add_argument("--concurrent", type=int, default=1,
                    help="realisations in flight per GPU (one context and stream each); the "
                         "per-kernel roofline timings then overlap")
    ap.add_argument("--inflight", type=int, default=2,
                    help="after the timed region (K = 1, one GPU, bond, launched march): the "
                         "same realisations again with this many in flight, reported as "
                         "in_flight (0 / 1: skip); never `value`")
    ap.add_argument("--march-mode", type=int, default=-1,
                    help="perc_set_march_mode bits (perc.h PERC_MARCH_*); -1: library default")
    ap.add_argument("--format", choices=("auto", "stencil", "stencil_tiled", "stencil_split", "csr"),
                    default="auto",
                    help="solver operator format (perc_set_matrix_format)")
    ap.add_argument("--inline-orders", action="store_true",
                    help="draw each timed realisation's occupation order inside the timed region "
                         "(host thread, overlapping the previous realisation's GPU solve) instead "
                         "of before it")
    ap.add_argument("--slabs", type=int, default=1,
                    help="row slabs of each CG solve on this GPU (perc_set_slabs; SURVEY §8(f) 2)")
    ap.add_argument("--cpu-worker", nargs=6, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--launch-stub", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="processes of the all-cores CPU ensemble baseline (0: the host CPU "
                         "share, at most 16; -1: skip)")
    args = ap.parse_args()
    if args.cpu_worker:
        return cpu_worker(args.cpu_worker, args.cpu_iters)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started here (the driver may call bench.py
        # --gpus N directly instead of through torch.distributed.run)
        return launch_ranks(args.gpus, sys.argv[1:], stub=args.launch_stub)
    if args.launch_stub:
        return launch_stub()
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        log("bench.py --gpus %d under a launcher with WORLD_SIZE=%s" % (args.gpus,
                                                                         os.environ["WORLD_SIZE"]))
        return 2

    import torch
    import torch.distributed as dist

    import percolation_amd as P
    from percolation_amd import api, ensemble

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or args.force_dist
    if use_dist:
        dist.init_process_group("nccl", device_id=dev)

    L_, p = args.L, args.p
    lat = 0 if args.lattice == "square" else 1
    nb = api.nbonds(lat, L_, L_, 0)
    t_sites = L_ * L_
    tb = int(p * nb)  # bondc.f:191
    if args.kind == "site":
        tb = 0
    elif args.kind == "sitebond":
        ts = int(args.ps * t_sites)
    if args.kind == "site":
        ts = int(p * t_sites)
    nreal = args.warmup + args.steps
    # tseed(ii) as bond_cond.f:65-70 generates them; never reused (the
    # reference's 1000 are extended with the same stream when needed)
    seeds = api.trial_seeds(args.master, max(1000, nreal * world))
    # inputs: occupation orders generated on the host and made resident in
    # HBM before the timed region.  "reference": the REAL*4 Fisher-Yates with
    # gfortran rand (bondc.f:162-174) -- for nb > 2^22 bonds its 22-bit
    # rand and float32 index arithmetic bias the order (hazard H10: at
    # L=4096 the top half of the lattice ends up ~39% occupied at pb=0.6 and
    # nothing spans), so the metric workload draws a uniform permutation
    # (numpy PCG64 seeded by tseed(ii)); the drop-in drivers keep the
    # reference RNG.
    t0 = time.perf_counter()
    orders, site_orders, ii_list, host_orders = [], [], [], []

    def draw(n, cnt, seed, salt=0):
        if args.occupancy == "reference":
            return api.shuffled_ids(n, seed)[:cnt]
        rng = np.random.default_rng([seed, salt] if salt else seed)
        return (rng.permutation(n)[:cnt] + 1).astype(np.int32)

    t_draw = 0.0
    inline = args.inline_orders and args.kind == "bond" and args.concurrent <= 1
    devocc = args.occupancy == "device"
    for k, ii in enumerate(ensemble.trial_indices(nreal, world, rank, nseeds=len(seeds))):
        if devocc:  # drawn on the GPU inside the realisation
            orders.append(None)
            site_orders.append(None)
            host_orders.append(None)
            ii_list.append(ii)
            continue
        if inline and k >= args.warmup and k != args.warmup:
            orders.append(None)  # drawn in the timed region (k == warmup: host copy kept below)
            host_orders.append(None)
            ii_list.append(ii)
            continue
        td = time.perf_counter()
        o = draw(nb, tb, int(seeds[ii])) if args.kind != "site" else np.zeros(1, np.int32)
        t_draw += time.perf_counter() - td
        if inline and k == args.warmup:  # drawn again inside the timed region
            orders.append(None)
            host_orders.append(o)
            ii_list.append(ii)
            continue
        orders.append(torch.from_numpy(np.ascontiguousarray(o)).to(dev))
        if args.kind != "bond":
            td = time.perf_counter()
            so = draw(t_sites, ts, int(seeds[ii]), salt=1)
            t_draw += time.perf_counter() - td
            site_orders.append(torch.from_numpy(np.ascontiguousarray(so)).to(dev))
        host_orders.append(o if k == args.warmup else None)
        ii_list.append(ii)
    torch.cuda.synchronize()
    log("rank %d: %d orders (nb=%d, tbonds=%d) in %.1fs" % (rank, nreal, nb, tb,
                                                            time.perf_counter() - t0))
    # the CPU baseline runs on two host cores of its own while the GPU
    # realisations run: the sample at L (same realisation as the first timed
    # one) and one whole L = 1024 solve as a measured anchor
    anchors = {}
    if (rank == 0 and world == 1 and not args.no_cpu_baseline and args.kind == "bond" and lat == 0
            and args.occupancy in ("uniform", "device")):
        anchors["sample"] = cpu_anchor_start(L_, p, int(seeds[ii_list[args.warmup]]), args.cpu_iters,
                                             args.occupancy)
        anchors["L1024"] = cpu_anchor_start(1024, p, int(seeds[0]), 0, args.occupancy)
    K = max(1, args.concurrent)

    def make_ctx():
        c = api.Context(lat, L_, L_, 0, device=local)
        c.set_matrix_format({"auto": P.FMT_AUTO, "stencil": P.FMT_STENCIL,
                             "stencil_tiled": P.FMT_STENCIL_TILED,
                             "stencil_split": P.FMT_STENCIL_SPLIT, "csr": P.FMT_CSR}[args.format])
        c.set_full_voltages(args.full_voltages)
        mode = args.march_mode if args.march_mode >= 0 else P.MARCH_DEFAULT
        if K > 1:  # no concurrent cooperative (resident) launches
            mode &= ~P._lib.SOLVE_RESIDENT
        c.set_march_mode(mode)
        if args.slabs > 1:
            c.set_slabs(args.slabs)
        return c

    # K contexts (each its own HIP stream): K realisations in flight per GPU
    ctxs = [make_ctx() for _ in range(K)]
    ctx = ctxs[0]
    N, nnz = ctx.system_size()

    seen = {}  # solver of a realisation that spanned (the last one may not)

    def note_solver(c, r):
        if r.get("nspan", 0) > 0 and "fmt" not in seen:
            try:
                seen["fmt"], seen["minfo"] = c.matrix_format(), c.march_info()
            except P.PercError:
                pass
        return r

    def run(k, ctx=ctx):
        return note_solver(ctx, run_(k, ctx))

    def run_(k, ctx):
        if devocc:  # occupancy drawn on the device (perc_occupy_random), then the path
            kind = {"bond": P._lib.BOND, "site": P._lib.SITE, "sitebond": P._lib.SITEBOND}[args.kind]
            rule = {"bond": P._lib.RULE_BOND, "site": P._lib.RULE_SITE,
                    "sitebond": P._lib.RULE_MIXED}[args.kind]
            cur = P._lib.CUR_FORTRAN if args.kind == "bond" else P._lib.CUR_MATLAB
            t_0 = time.perf_counter()
            ctx.occupy_random(kind, ts if args.kind != "bond" else 0, tb, int(seeds[ii_list[k]]))
            li = ctx.label()
            t_1 = time.perf_counter()
            if li["nspan"] == 0:
                return dict(gtop=0.0, gbot=0.0, iter=0, nspan=0, t_label_ms=(t_1 - t_0) * 1e3,
                            t_solve_ms=0.0, t_total_ms=(t_1 - t_0) * 1e3)
            c = ctx.conductance(rule, cur, tol=args.tol, itmax=args.itmax)
            t_2 = time.perf_counter()
            return dict(gtop=c["gtop"], gbot=c["gbot"], iter=c["iter"], nspan=li["nspan"],
                        t_label_ms=(t_1 - t_0) * 1e3, t_solve_ms=c["t_solve_ms"],
                        t_total_ms=(t_2 - t_0) * 1e3)
        if args.kind == "bond":
            return ctx.bondc_realisation(None, tb, tol=args.tol, itmax=args.itmax,
                                         device_ptr=orders[k].data_ptr())
        # ConductCalc.m site / mixed rules (MATLAB/ConductCalc.m:88-165)
        kind = P._lib.SITE if args.kind == "site" else P._lib.SITEBOND
        t_0 = time.perf_counter()
        ctx.occupy_device(kind, site_orders[k].data_ptr(), ts,
                          orders[k].data_ptr() if kind == P._lib.SITEBOND else None, tb)
        li = ctx.label()
        t_1 = time.perf_counter()
        c = ctx.conductance(P._lib.RULE_SITE if args.kind == "site" else P._lib.RULE_MIXED,
                            P._lib.CUR_MATLAB, tol=args.tol, itmax=args.itmax)
        t_2 = time.perf_counter()
        return dict(gtop=c["gtop"], gbot=c["gbot"], iter=c["iter"], nspan=li["nspan"],
                    t_label_ms=(t_1 - t_0) * 1e3, t_solve_ms=c["t_solve_ms"],
                    t_total_ms=(t_2 - t_0) * 1e3)

    for k in range(args.warmup):
        r = run(k, ctxs[k % K])
        log("warmup %d: iter=%d Gtop=%.12g %.0f ms" % (k, r["iter"], r["gtop"], r["t_total_ms"]))
    for c in ctxs:
        c.set_kernel_timing(True)
        c.kernel_stats(reset=True)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timed = list(range(args.warmup, nreal))
    if inline:
        # order k + 1 is drawn and uploaded by a host thread while
        # realisation k solves (libperc calls release the GIL); the first
        # timed order is drawn inside the timed region too
        from concurrent.futures import ThreadPoolExecutor

        def prep(k_):
            torch.cuda.set_device(local)
            o_ = draw(nb, tb, int(seeds[ii_list[k_]]))
            return torch.from_numpy(np.ascontiguousarray(o_)).to(dev)

        results = []
        with ThreadPoolExecutor(1) as tp:
            fut = tp.submit(prep, timed[0])
            for j_, k in enumerate(timed):
                orders[k] = fut.result()
                if j_ + 1 < len(timed):
                    fut = tp.submit(prep, timed[j_ + 1])
                results.append(run(k))
    elif K == 1:
        results = [run(k) for k in timed]
    else:  # one host thread per context (ctypes drops the GIL in libperc calls)
        from concurrent.futures import ThreadPoolExecutor
        lanes = [[k for k in timed if (k - args.warmup) % K == ci] for ci in range(K)]
        with ThreadPoolExecutor(K) as pool:
            futs = [pool.submit(lambda ks_, c_: [run(k_, c_) for k_ in ks_], lanes[ci], ctxs[ci])
                    for ci in range(K)]
            per = [f.result() for f in futs]
        results = [per[(k - args.warmup) % K][(k - args.warmup) // K] for k in timed]
    for k, r in zip(timed, results):
        log("step %d (ii=%d): nspan=%d iter=%d Gtop=%.12g Gbot=%.12g label %.0f ms solve %.0f ms "
            "total %.0f ms" % (k - args.warmup, ii_list[k] + 1, r["nspan"], r["iter"], r["gtop"],
                               r["gbot"], r["t_label_ms"], r["t_solve_ms"], r["t_total_ms"]))
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ks = ctx.kernel_stats(reset=True)
    for c in ctxs[1:]:
        for key_, v_ in c.kernel_stats(reset=True).items():
            ks[key_] += v_
    # ensemble statistics: the only collective (RCCL all-reduce over xGMI)
    stats, tmax = ensemble.allreduce(ensemble.local_stats(results), elapsed, device=dev)
    # solves/s = realisations completed per second end to
    # end (labeling + spanning test, and assembly + CG + currents when a
    # cluster spans); the CG solves among them are reported separately
    nsolves = int(stats[0])
    nspan = int(stats[3])
    value = nsolves / tmax

    fmt_names = {P.FMT_STENCIL: "stencil", P.FMT_STENCIL_TILED: "stencil_tiled",
                 P.FMT_STENCIL_SPLIT: "stencil_split", P.FMT_CSR: "csr"}
    try:  # the format the solves used (the last realisation may not span: no system)
        fmt = fmt_names[ctx.matrix_format()]
        assembled = True
        minfo = ctx.march_info()
    except P.PercError:
        minfo = dict(kernel="none", qfree=False)
        fmt = {"auto": "stencil"}.get(args.format, args.format)
        assembled = False
    if "fmt" in seen:  # what the spanning realisations ran (labels + bytes below)
        fmt, minfo = fmt_names[seen["fmt"]], seen["minfo"]
    minfo["strips"] = bool(minfo.get("strips")) and args.slabs <= 1

    def kernel_set(f, probe=False):
        """(key, stats key, perc_bench_kernel id, bytes) of the CG kernels of
        operator format f"""
        full = args.full_voltages
        if f in ("stencil", "stencil_tiled") and minfo.get("kernel") == "resident" and not probe:
            # whole iterations in one persistent launch, r / q / codes held
            # on chip: the bytes are the streaming-equivalent 52 B/row (what
            # the launched march P + B move per iteration, 26N each) plus the
            # electrode-adjacent x rows -- "how fast against the streaming
            # solver's traffic"; the floor under it is the measured grid
            # synchronisation (roofline.sync_floor_ms, perc_bench_kernel 6)
            return [("res", "spmv", 5, 52 * N + x_bytes(N, L_, full))]
        if f in ("stencil", "stencil_tiled"):
            qf = f == "stencil" and minfo["qfree"]
            if f == "stencil" and not qf and minfo.get("kernel") == "wave":
                # the march kernels carry no x: the streaming B applies
                # x += ak p(k) (reads x and p(k), writes x: 24 B per x row)
                xb = 24 * N if full else 24 * 2 * L_
                return [("pm", "spmv", 1, 34 * N), ("resid", "resid", 2, resid_bytes(N, f) + xb)]
            if qf and minfo.get("strips"):
                # strip-major q-free march: x += ak p(k) in the march B; per
                # element each kernel reads p, r and the row code and writes
                # one vector: 24 B + the code (2 B u16, 0.5 B nibble codes)
                xb = 24 * N if full else 24 * 2 * L_
                cb = 0.5 if minfo.get("nibble") else 2.0
                return [("pm", "spmv", 1, int((24 + cb) * N)), ("resid", "resid", 2, int((24 + cb) * N) + xb)]
            return [("pm" if f == "stencil" else "ps", "spmv", 1, ps_bytes(N, L_, full, qf)),
                    ("resid", "resid", 2, resid_bytes(N, f))]
        return [("spmv", "spmv", 1, spmv_bytes(N, nnz, f)), ("resid", "resid", 2, resid_bytes(N, f)),
                ("xp", "xp", 3, xp_bytes(N, f, L_, full))]

    # per-kernel live timing: HIP events on the context stream around the
    # launches of every 64th CG iteration of the timed realisations (those
    # that did work; perc_set_kernel_timing -- a timed launch's event packets
    # open a dispatch gap of several us, so every 8th cost the solve ~1 %)
    kern = {}
    for key, skey, _, nbytes in kernel_set(fmt):
        n_ = max(ks[skey + "_n"], 1)
        avg = ks[skey + "_ms"] / n_
        kern[key] = {"kernel": kernel_label(key, minfo), "avg_launch_ms": round(avg, 5),
                     "launches": ks[skey + "_n"], "total_ms": round(ks[skey + "_ms"], 1),
                     "bytes_per_launch": nbytes,
                     "gbs": round(nbytes / (avg * 1e-3) / 1e9, 1) if avg > 0 else None}
    # the roofline line is the kernel with the most device time
    dom = max(kern, key=lambda k_: kern[k_]["total_ms"])
    traffic, traffic_src = pmc_traffic(rocprof_base(dom, fmt, minfo), L_, args.kind)
    rp_ms, rp_src = rocprof_avg(rocprof_base(dom, fmt, minfo), L_)
    achieved = kern[dom]["gbs"] or 0.0  # 0: no realisation spanned, nothing solved
    iter_ms = sum(v["avg_launch_ms"] for v in kern.values())
    iter_bytes = sum(v["bytes_per_launch"] for v in kern.values())
    # after the timed region, on the last assembled system: each kernel in
    # both operator formats, back to back (perc_bench_kernel; clobbers x)
    probe = {}
    for fname, fcode in (("stencil", P.FMT_STENCIL), ("stencil_tiled", P.FMT_STENCIL_TILED),
                         ("stencil_split", P.FMT_STENCIL_SPLIT),
                         ("csr", P.FMT_CSR)) if assembled else ():
        try:
            ctx.set_matrix_format(fcode)
        except Exception:
            continue
        row = {}
        plain = [] if fname in ("stencil", "stencil_tiled") else [("spmv_plain", "", 0, spmv_bytes(N, nnz, fname))]
        for key, _, which, nbytes in plain + kernel_set(fname, probe=True):
            ms = ctx.bench_kernel(which, 50)
            row[key] = {"ms": round(ms, 5), "gbs": round(nbytes / (ms * 1e-3) / 1e9, 1)}
        probe[fname] = row
    sync_floor = None
    if minfo.get("kernel") == "resident" and assembled:
        # two block sums + two tagged-granule all-gathers per iteration on
        # the resident grid, nothing else (k_res_sync_probe)
        sync_floor = round(ctx.bench_kernel(6, 20), 5)
    labeling = None
    if devocc and rank == 0:
        labeling = labeling_probe(ctx, P, L_, nb, tb, [int(seeds[ii_list[k]]) for k in timed][:4],
                                  args.kind, ts if args.kind != "bond" else 0)
    # realisations in flight (one context and stream each): what a throughput
    # run of the ensemble gets from one GPU -- the march kernels' fixed costs
    # (ramp, walk-end spread, reduction tail) of one solve are filled by the
    # other's work.  Reported beside `value` (K = 1), whose per-kernel
    # roofline it would blur.
    in_flight = None
    if (args.inflight > 1 and K == 1 and world == 1 and devocc and args.kind == "bond"
            and minfo.get("kernel") != "resident" and timed):
        K2 = args.inflight
        mode0 = args.march_mode if args.march_mode >= 0 else P.MARCH_DEFAULT
        pool_ctx = [ctx] + [make_ctx() for _ in range(K2 - 1)]
        for c in pool_ctx:
            c.set_march_mode(mode0 & ~P._lib.SOLVE_RESIDENT)
            c.set_kernel_timing(False)
        ks2 = (timed * (2 * K2))[:2 * K2]
        from concurrent.futures import ThreadPoolExecutor
        lanes2 = [[k for j, k in enumerate(ks2) if j % K2 == ci] for ci in range(K2)]
        torch.cuda.synchronize()
        t_if = time.perf_counter()
        with ThreadPoolExecutor(K2) as pool:
            futs = [pool.submit(lambda ks_, c_: [run_(k_, c_) for k_ in ks_], lanes2[ci], pool_ctx[ci])
                    for ci in range(K2)]
            res2 = [r_ for f in futs for r_ in f.result()]
        torch.cuda.synchronize()
        t_if = time.perf_counter() - t_if
        for c in pool_ctx[1:]:
            c.close()
        ctx.set_march_mode(mode0)
        in_flight = {"k": K2, "realisations": len(ks2), "value": round(len(ks2) / t_if, 5),
                     "unit": "solves/s", "ms_per_step": round(t_if / len(ks2) * 1e3, 2),
                     "cg_iterations_mean": round(float(np.mean([r_["iter"] for r_ in res2])), 1),
                     "note": "the timed realisations again, %d in flight (one context and stream "
                             "each), after the timed region; not `value`" % K2}
    copy_ms = ctx.bench_kernel(4, 20)
    copy_bytes = 2 * 8 * (64 << 20)  # 512 MB read + 512 MB written (perc_bench_kernel 4)
    stream_copy = {"ms": round(copy_ms, 5), "bytes": copy_bytes,
                   "gbs": round(copy_bytes / (copy_ms * 1e-3) / 1e9, 1)}

    out = {
        "metric": "CG SpMV GB/s + conductance solves/sec, L=4096 square lattice at p=0.60",
        "value": round(value, 5),
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(tmax / max(args.steps, 1) * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: %s occupation of int(p*nb) bonds per realisation, seeds "
                 "tseed(ii) from master %d (bond_cond.f:65-70)"
                 % ({"device": "uniform, drawn on the GPU inside the timed realisation "
                               "(perc_occupy_random: counter-based keys, radix select)",
                     "uniform": "uniform PCG64 order drawn on the host before the timed region,"
                                " resident in HBM",
                     "reference": "reference REAL*4 gfortran-rand Fisher-Yates order"}
                    [args.occupancy], args.master)),
        "config": {"workload": (
            "%s L=%d bond percolation p=%.2f, bondc semantics" % (args.lattice, L_, p)
            if args.kind == "bond" else
            "%s L=%d site percolation p=%.3f, ConductCalc site rule" % (args.lattice, L_, p)
            if args.kind == "site" else
            "%s L=%d mixed ps=%.3f pb=%.3f, ConductCalc mixed rule" % (args.lattice, L_, args.ps, p))
            + " (labeling+assembly+Jacobi-PCG tol %g itol 2+currents)" % args.tol,
                   "lattice": args.lattice, "kind": args.kind,
                   "L": L_, "p": p, "rows": N, "nnz_offdiag": nnz,
                   "full_voltages": bool(args.full_voltages), "parallelism":
                   "realisations sharded over %d GPU(s), RCCL stats all-reduce" % world,
                   "concurrent_per_gpu": K, "slabs": args.slabs},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                     "achievable": stream_copy["gbs"],
                     "frac_of_achievable": round(achieved / stream_copy["gbs"], 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "avg_launch_ms_rocprof": rp_ms, "rocprof_source": rp_src,
                     "timing_note": "avg_launch_ms: every 64th launch timed live by its own "
                                    "dispatch timestamps (hipExtLaunchKernel events on the "
                                    "context stream); a timed launch carries the events' "
                                    "cache write-back, so it reads a few % above the "
                                    "kernel-trace average of all launches "
                                    "(avg_launch_ms_rocprof, committed rocprofv3 --stats)",
                     "kernel": kern[dom]["kernel"], "format": fmt,
                     "bytes_per_launch": kern[dom]["bytes_per_launch"],
                     "avg_launch_ms": kern[dom]["avg_launch_ms"],
                     "launches": kern[dom]["launches"],
                     **({"note": "%d realisations in flight per GPU: kernel durations overlap"
                                 % K} if K > 1 else {}),
                     **({"bytes_model": "streaming-equivalent 52 B/row/iteration (resident "
                                        "solve: r, q, codes on chip)",
                         "sync_floor_ms": sync_floor,
                         "sync_floor_frac": round(sync_floor / kern[dom]["avg_launch_ms"], 3)
                         if kern[dom]["avg_launch_ms"] else None}
                        if sync_floor is not None else {})},
        "realisations_per_s": round(value, 5),
        "cg_solves_per_s": round(nspan / tmax, 5),
        "cg_solves": nspan,
        "cg_iterations_mean": round(float(stats[4]) / max(nspan, 1), 1),
        "spanning_fraction": round(float(stats[3]) / max(nsolves, 1), 3),
        "host_order_ms_per_realisation": round(t_draw * 1e3 / max(nreal, 1), 1),
        "orders_in_timed_region": bool(inline or devocc),
        "host_order_note": (
            "occupancy drawn on the GPU inside each timed realisation (no host order)" if devocc
            else "orders drawn on a host thread inside the timed region, overlapping the "
                 "previous realisation's solve" if inline
            else "occupation orders are drawn on the host before the timed region and kept in "
                 "HBM; an ensemble that draws them inline pays this per realisation on one host "
                 "core unless it overlaps the GPU solve"),
        "gtop_mean": float(stats[1]) / max(nsolves, 1),
        "cg_iteration": {"ms": round(iter_ms, 5), "bytes": iter_bytes,
                         "gbs": round(iter_bytes / (iter_ms * 1e-3) / 1e9, 1) if iter_ms > 0
                         else None},
        "cg_kernels": kern,
        "kernel_probe": probe,
        "stream_copy": stream_copy,
    }
    if labeling is not None:
        out["labeling"] = labeling
    if in_flight is not None:
        out["in_flight"] = in_flight
    if rank == 0 and world == 1 and args.kind == "bond" and devocc:
        out["pcie_inclusive"] = {"note": "occupancy drawn on the device: no host array crosses "
                                         "PCIe per realisation"}
    if rank == 0 and world == 1 and args.kind == "bond" and host_orders[args.warmup] is not None:
        # the host-array boundary (perc_occupy with a host order) adds one
        # PCIe upload of the order per realisation; timed here outside the
        # metric: host-order occupy + label vs device-order occupy + label
        ho = host_orders[args.warmup]

        def occ_label(host):
            torch.cuda.synchronize()
            t_ = time.perf_counter()
            if host:
                ctx.occupy(P._lib.BOND, bond_order=ho, nbonds_=tb)
            else:
                ctx.occupy_device(P._lib.BOND, None, 0, orders[args.warmup].data_ptr(), tb)
            ctx.label()
            return time.perf_counter() - t_

        occ_label(True)
        th = min(occ_label(True) for _ in range(3))
        td = min(occ_label(False) for _ in range(3))
        up_s = max(th - td, 0.0)
        out["pcie_inclusive"] = {
            "upload_bytes": int(ho.nbytes), "upload_ms": round(up_s * 1e3, 3),
            "value": round(nsolves / (tmax + up_s * nsolves), 5), "unit": "solves/s",
            "note": "host-order boundary: value with one H2D upload of the occupation "
                    "order per realisation (occupy+label host minus device, best of 3)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.kind == "bond" and lat == 0:
        log("cpu baseline: waiting for the oracle processes ...")
        try:
            if "sample" in anchors:
                out["cpu_baseline"] = cpu_anchor_finish(anchors["sample"], results[0]["iter"])
                out["cpu_baseline"]["anchor_L1024"] = cpu_anchor_finish(anchors["L1024"])
            else:  # reference-order occupancy: the sample in this process
                ho = host_orders[args.warmup]
                out["cpu_baseline"] = cpu_baseline(L_, p, ho, results[0]["iter"], args.cpu_iters)
        except Exception as e:  # keep the GPU line even if the host is short of memory
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
        if args.cpu_cores >= 0 and args.occupancy in ("uniform", "device"):
            try:
                aff = len(os.sched_getaffinity(0))
            except AttributeError:
                aff = os.cpu_count() or 1
            cores = args.cpu_cores or max(1, min(16, aff, int(os.environ.get("OMP_NUM_THREADS", "16"))))
            log("cpu ensemble baseline: %d processes ..." % cores)
            iters_mean = int(round(np.mean([r["iter"] for r in results])))
            ens_seeds = [int(seeds[(ii_list[args.warmup] + j) % len(seeds)]) for j in range(cores)]
            try:
                out["cpu_baseline_ensemble"] = cpu_ensemble(L_, p, ens_seeds, iters_mean, nb, tb,
                                                            args.cpu_ensemble_iters, cores,
                                                            args.occupancy)
            except Exception as e:
                out["cpu_baseline_ensemble"] = {"value": None, "error": repr(e)}
    for c in ctxs:
        c.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_dist:
        # (normal teardown: libperc binds to torch's HIP / HSA / RCCL copies,
        # one runtime per process -- percolation_amd/_lib.py _one_runtime)
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
