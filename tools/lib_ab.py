#!/usr/bin/env python3
"""Same-box A/B of libperc probe builds (percolation_amd/probe/libperc_<tag>.so,
`make -C percolation_amd/csrc probe TAG=... PFLAGS=...`) against the
in-tree library: per library, in a child process of its own (PERC_LIBPERC),
the libraries alternating for `rounds` rounds, each figure its best.

--what solve: one L x L bond realisation (--kind sitebond --ps: a mixed one,
  ConductCalc's mixed rule), perc_bench_kernel 1 (P), 2 (B) and
  5 (a whole iteration), best of 3 x `reps` launches, plus ms per iteration
  of fixed-iteration solves (slope between itmax/2 and itmax, tol 0);
  --format csr: the CSR operator (0 plain SpMV, 1 S, 2 B, 3 P, 5 iteration);
--what label: per realisation (device-drawn occupancy, `reps`
  realisations; --kind bond, or sitebond with --ps: config 5's mixed
  kind), wall ms of perc_occupy_random, perc_label (labels + spanning test
  + its read-back) and the partition's cluster count.

  python tools/lib_ab.py --L 4096 --libs main,s16,s18 [--mode 1559]
  python tools/lib_ab.py --what label --L 4096 --libs main,mrows
  python tools/lib_ab.py --what label --L 8192 --kind sitebond --ps 0.593 --p 0.5 --libs main,r5f
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def child_label(args):
    import torch  # (torch.cuda.synchronize: a device-wide wait)
    from percolation_amd import _lib as PL
    from percolation_amd import api
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    occ, lab, fp = [], [], []
    with api.Context(0, L_, L_, 0) as ctx:
        for k in range(args.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if args.kind == "bond":
                ctx.occupy_random(PL.BOND, 0, int(args.p * nb), 1000 + k)
            else:
                ctx.occupy_random(PL.SITEBOND, int(args.ps * L_ * L_), int(args.p * nb), 1000 + k)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            li = ctx.label()
            t2 = time.perf_counter()
            if k:
                occ.append((t1 - t0) * 1e3)
                lab.append((t2 - t1) * 1e3)
            fp.append([li["nspan"], li["nclusters"]])
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(json.dumps(dict(fp=fp, occupy_ms=med(occ), label_ms=med(lab))), flush=True)


def child(args):
    from percolation_amd import _lib as PL
    from percolation_amd import api
    if args.what == "label":
        return child_label(args)
    L_ = args.L
    nb = api.nbonds(0, L_, L_, 0)
    out = {}
    with api.Context(0, L_, L_, 0) as ctx:
        if args.mode >= 0:
            ctx.set_march_mode(args.mode)
        for part in filter(None, args.wspec.split("/")):  # "which:w0,w1,w2/..."
            which, ws = part.split(":")
            ctx.set_band_weights(int(which), [int(x) for x in ws.split(",")])
        if args.kind == "bond":
            ctx.occupy_random(PL.BOND, 0, int(args.p * nb), 777)
            rule = (PL.RULE_BOND, PL.CUR_FORTRAN)
        else:  # ConductCalc's mixed rule (the config-5 companion's matrix)
            ctx.occupy_random(PL.SITEBOND, int(args.ps * L_ * L_), int(args.p * nb), 777)
            rule = (PL.RULE_MIXED, PL.CUR_MATLAB)
        assert ctx.label()["nspan"] > 0
        if args.format == "csr":
            ctx.set_matrix_format(PL.FMT_CSR)
        c = ctx.conductance(*rule, tol=1e-8, itmax=args.iters)
        out["fp"] = [c["iter"], c["gtop"], c["gbot"]]  # same numbers across store policies
        kset = ((1, "P"), (2, "B"), (5, "iteration")) if args.format == "default" else \
            ((0, "spmv_plain"), (1, "S"), (2, "B"), (3, "P"), (5, "iteration"))
        for w, k in kset:
            out[k] = min(ctx.bench_kernel(w, args.reps) for _ in range(3))
        t = {}
        for n in (args.iters // 2, args.iters):
            t0 = time.perf_counter()
            it = ctx.conductance(*rule, tol=0.0, itmax=n - 1)["iter"]
            t[n] = (time.perf_counter() - t0, it)
        (t1, i1), (t2, i2) = t[args.iters // 2], t[args.iters]
        out["solve_ms_per_it"] = (t2 - t1) * 1e3 / (i2 - i1)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=4096)
    ap.add_argument("--p", type=float, default=0.6)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--iters", type=int, default=600)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--mode", type=int, default=-1)
    ap.add_argument("--libs", default="main")
    ap.add_argument("--what", default="solve", choices=("solve", "label"))
    ap.add_argument("--kind", default="bond", choices=("bond", "sitebond"))
    ap.add_argument("--ps", type=float, default=0.593)
    ap.add_argument("--format", default="default", choices=("default", "csr"))
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--wspec", default="", help=argparse.SUPPRESS)
    ap.add_argument("--wsets", default="",
                    help="band-weight variants of the main library: 'name=which:w,w,w/which:w,w,w;...'")
    args = ap.parse_args()
    if args.child:
        return child(args)
    libs = [(lib, lib, "") for lib in args.libs.split(",")]
    for ws in filter(None, args.wsets.split(";")):
        name, spec = ws.split("=")
        libs.append((name, "main", spec))
    best = {}
    fps = {}
    for _ in range(args.rounds):
        for name, lib, spec in libs:
            env = dict(os.environ)
            if lib != "main":
                env["PERC_LIBPERC"] = os.path.join(REPO, "percolation_amd", "probe", "libperc_%s.so" % lib)
            cmd = [sys.executable, os.path.abspath(__file__), "--child", "--L", str(args.L), "--p", str(args.p),
                   "--reps", str(args.reps), "--iters", str(args.iters), "--mode", str(args.mode),
                   "--what", args.what, "--format", args.format, "--wspec", spec, "--kind", args.kind,
                   "--ps", str(args.ps)]
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                sys.stderr.write(r.stderr[-3000:])
                raise SystemExit("child %s failed rc=%d" % (name, r.returncode))
            o = json.loads(r.stdout.strip().splitlines()[-1])
            fps.setdefault(name, o.pop("fp"))
            b = best.setdefault(name, {})
            for k, v in o.items():
                b[k] = min(b.get(k, 9e9), v)
    out = {lib: {k: round(v, 5) for k, v in b.items()} for lib, b in best.items()}
    out["fingerprints"] = fps
    out["L"] = args.L
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
