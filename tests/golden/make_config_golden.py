#!/usr/bin/env python3
"""Conductance fixtures at the BASELINE config sizes, from the CPU oracle.

TEST INFRASTRUCTURE.  The reference itself stops at 50x50 (dense G, NMAX =
20000), so above that size the pin is the oracle's literal
restatement (oracle/perc_oracle.c), which tests/test_oracle_golden.py holds
bit-exact against the reference's own outputs at <= 64^2.  For each case
this script

  * rebuilds the occupation order from its recipe (the reference REAL*4
    shuffle seeded by tseed(ii) where N <= 2^22, else the uniform PCG64
    permutation bench.py uses -- hazard H10),
  * labels it with the oracle's O(N alpha) replay (reference label numbers)
    and picks the spanning cluster (bondc.f:413-456 / site.f:309-344),
  * assembles the interior system and runs the oracle's literal linbcg
    (bondc.f:750-838) at the reference tolerance 1e-8 and converged at
    1e-13, then the terminal currents (bondc.f:554-592 or ConductCalc.m),

and writes tests/golden/configs/<case>.json: the recipe, the partition
fingerprint (sha256 of the canonical min-site id per site), Gtop, Gbot,
iter, err and a decimated err history for both tolerances.

Round 3 (--decades): the same iterates from one threaded run
(or_linbcg_sym: bitwise the literal linbcg's on a symmetric system, checked
against every solve the literal runs committed) with x snapshotted at
1e-8 ... 1e-17, so each fixture carries its own convergence: the change of
Gtop / Gbot over the last decades shows where the oracle has converged.

Usage: python tests/golden/make_config_golden.py [case ...]   (CPU, minutes to hours)
       GOLDEN_THREADS=k python tests/golden/make_config_golden.py --decades [case ...]
       GOLDEN_TOLS=1e-8,1e-9 GOLDEN_PREFIX=2000 GOLDEN_THREADS=6 \
           python tests/golden/make_config_golden.py --decades c5c_sq8192_mixed_p85_dev
       GOLDEN_THREADS=k python tests/golden/make_config_golden.py --assoc [case ...]
       GOLDEN_THREADS=k python tests/golden/make_config_golden.py --assoc-tree [case ...]
"""
import hashlib
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
OUT = os.path.join(HERE, "configs")
OUT_LARGE = os.path.join(HERE, "large")

MASTER = 58302  # bench.py / Square/bond_cond.f:65-70 master seed

# case -> recipe.  order: "ref" = srand(tseed) + REAL*4 shuffle (bondc.f:162-174),
# "pcg64" = numpy default_rng(tseed).permutation (bench.py --occupancy uniform)
CASES = {
    # BASELINE config 2: 1024^2 square bond at p_c = 0.5
    "c2_sq1024_bond_p50": dict(lattice=0, L=1024, kind="bond", p=0.50, order="ref"),
    # BASELINE config 3: 1024^2 triangular site at 0.5, ConductCalc site rule
    "c3_tri1024_site_p50": dict(lattice=1, L=1024, kind="site", p=0.50, order="ref"),
    # BASELINE config 4's per-GPU shape: 2048^2 square bond at 0.5
    "c4_sq2048_bond_p50": dict(lattice=0, L=2048, kind="bond", p=0.50, order="pcg64"),
    # the metric: 4096^2 square bond at 0.6 (bench.py's first realisation)
    "metric_sq4096_bond_p60": dict(lattice=0, L=4096, kind="bond", p=0.60, order="pcg64"),
    # config 5's rule at a size the oracle solves: 1024^2 square mixed site-then-bond at
    # ps = pb = 0.85 (spans; config 5's (0.593, 0.5) does not), the reference shuffles with
    # sitebond.f's own seeds (sseed 143285 sites, bseed 43716 bonds; sitebond.f:129-189),
    # ConductCalc.m:134-160 mixed rule
    "c5m_sq1024_mixed_p85": dict(lattice=0, L=1024, kind="mixed", p=0.85, pb=0.85,
                                 order="ref", sseed=143285, bseed=43716),
    # the realisation bench.py times first: 4096^2 square bond at 0.6, occupancy drawn on the
    # GPU by perc_occupy_random with tseed(ii = 2) (the host restatement perc_random_order
    # gives the same ids, tests/test_labeling_oracle.py; round 4)
    "bench_sq4096_bond_p60_dev": dict(lattice=0, L=4096, kind="bond", p=0.60, order="device",
                                      ii=2),
    # config 5's near-critical companion at its own size (round 6): 8192^2 square mixed
    # site-then-bond at ps = pb = 0.85, both occupations drawn on the GPU by
    # perc_occupy_random(PERC_SITEBOND, seed 777) as tools/l8192_probe.py does (host
    # restatement perc_random_order), ConductCalc.m:134-160 mixed rule; vectors past the
    # Infinity Cache, so the production solver is the ROW-MAJOR q-free march.  Kept in
    # tests/golden/large/ (decades 1e-8, 1e-9 and the complete err history of the first
    # GOLDEN_PREFIX iterations; not a converged fixture): tests/test_large_fixture.py
    "c5c_sq8192_mixed_p85_dev": dict(lattice=0, L=8192, kind="mixed", p=0.85, pb=0.85,
                                     order="device", seed=777),
}
LARGE = {"c5c_sq8192_mixed_p85_dev"}  # written to tests/golden/large/
TOLS = (1e-8, 1e-13, 1e-14)
# --decades: one threaded run of the same iterates (oracle or_linbcg_sym, bitwise the
# literal linbcg's on these symmetric systems) snapshotting x at every tolerance here
TOLS_DECADES = tuple(float(t) for t in os.environ.get(
    "GOLDEN_TOLS", "1e-8,1e-13,1e-14,1e-15,1e-16,1e-17").split(","))
HIST_EVERY = 256
# re-associated reference solvers (or_linbcg_sym dot_order): reversed serial sums,
# pairwise (tree) sums, serial sums of 4096 contiguous blocks then of the block sums
ASSOC_KEYS = {1: "assoc_desc", 2: "assoc_tree", 3: "assoc_block"}
ASSOC_FLAGS = {"--assoc": 1, "--assoc-tree": 2, "--assoc-block": 3}


def _oracle():
    import oracle_lib as O
    return O


def bond_pairs(O, lattice, L, recipe_order, seed, p):
    b1, b2 = O.bond_list(lattice, L, L, 0)
    nb = len(b1)
    tb = int(p * nb)
    if recipe_order == "ref":
        _, _, o1, o2 = O.bond_order(lattice, L, L, 0, seed)
    elif recipe_order == "device":  # perc_occupy_random's ids (host restatement)
        sys.path.insert(0, REPO)
        from percolation_amd import _lib as PL, api
        ids = api.random_order(nb, tb, seed, PL.BOND).astype(np.int64) - 1
        o1, o2 = O.i32(nb + 1), O.i32(nb + 1)
        o1[:tb], o2[:tb] = b1[ids], b2[ids]
    else:
        ids = np.random.default_rng(seed).permutation(nb)[:tb]
        o1, o2 = O.i32(nb + 1), O.i32(nb + 1)
        o1[:tb], o2[:tb] = b1[ids], b2[ids]
    return b1, b2, o1, o2, tb


def canon_hash(canon):
    return hashlib.sha256(np.ascontiguousarray(canon, dtype=np.int32).tobytes()).hexdigest()


def canon_from_bonds(b1, b2, label, t):
    canon = np.zeros(t, np.int64)
    lab = label.astype(np.int64)
    occ = lab > 0
    mins = np.full(lab.max() + 1, np.iinfo(np.int64).max)
    np.minimum.at(mins, lab[occ], b1[occ])
    for arr in (b1, b2):
        np.maximum.at(canon, arr[occ] - 1, mins[lab[occ]])
    return canon


def canon_from_sites(s):
    t = len(s)
    canon = np.zeros(t, np.int64)
    occ = s > 0
    mins = np.full(s.max() + 1, np.iinfo(np.int64).max)
    sites = np.arange(1, t + 1)
    np.minimum.at(mins, s[occ], sites[occ])
    canon[occ] = mins[s[occ]]
    return canon


def label_case(rc, seed):
    """Occupy + oracle replay + spanning; returns (dict, system inputs) or None."""
    O = _oracle()
    lib = O.lib()
    lattice, L = rc["lattice"], rc["L"]
    t = L * L
    if rc["kind"] == "bond":
        b1, b2, o1, o2, tb = bond_pairs(O, lattice, L, rc["order"], seed, rc["p"])
        nb = len(b1)
        label, csize = O.i32(nb), O.i32(nb + 2)
        import ctypes as C
        mx, ms = C.c_int(), C.c_int()
        cln = lib.or_label_bonds_replay(lattice, L, L, 0, nb, b1, b2, o1, o2, tb, label, csize,
                                        C.byref(mx), C.byref(ms))
        perccln = lib.or_span_bonds(L, L, nb, b1, b2, label, csize, cln)
        if perccln <= 0:
            return None
        canon = canon_from_bonds(b1, b2, label, t)
        gval = O.f64(nb)
        lib.or_bond_values(0, nb, b1, b2, label, O.i32(1), perccln, 1.0, 1e-12, gval)
        info = dict(occupied=tb, cln=cln, maxcs=ms.value, perccln=perccln,
                    perccls=int(csize[perccln]), span_sites=int(np.sum(canon == canon[
                        b1[np.argmax(label == perccln)] - 1])))
        sysin = dict(b1=b1, b2=b2, gval=gval, rhs_rule=0, cur_rule=0, cur_thresh=1e-10)
    elif rc["kind"] == "mixed":
        if rc["order"] == "device":  # perc_occupy_random(PERC_SITEBOND, seed): host restatement
            sys.path.insert(0, REPO)
            from percolation_amd import _lib as PL, api
            b1, b2 = O.bond_list(lattice, L, L, 0)
            nb = len(b1)
            ts, tb = int(rc["p"] * t), int(rc["pb"] * nb)
            so = O.i32(t + 1)
            so[:ts] = api.random_order(t, ts, rc["seed"], PL.SITE)
            ids = api.random_order(nb, tb, rc["seed"], PL.BOND).astype(np.int64) - 1
            o1, o2 = O.i32(nb + 1), O.i32(nb + 1)
            o1[:tb], o2[:tb] = b1[ids], b2[ids]
        else:
            b1, b2, o1, o2 = O.bond_order(lattice, L, L, 0, rc["bseed"])
            nb = len(b1)
            so = O.site_order(t, rc["sseed"])
            ts, tb = int(rc["p"] * t), int(rc["pb"] * nb)
        s, bl, csize, cln, maxcn, maxcs = O.label_sitebond(lattice, L, L, 0, b1, b2, so, ts, o1,
                                                           o2, tb, literal=False)
        perccln = lib.or_span_sites(L, L, s, csize, cln, 2 * L - 1)
        if perccln <= 0:
            return None
        canon = canon_from_sites(s)
        gval = O.f64(nb)
        lib.or_bond_values(2, nb, b1, b2, bl, s, perccln, 1.0, 1e-12, gval)
        info = dict(occupied_sites=ts, occupied_bonds=tb, cln=cln, maxcs=maxcs, perccln=perccln,
                    perccls=int(csize[perccln]), span_sites=int(np.sum(s == perccln)),
                    g0_bonds=int(np.sum(gval == -1.0)))
        sysin = dict(b1=b1, b2=b2, gval=gval, rhs_rule=0, cur_rule=1, cur_thresh=0.0)
    else:
        order = O.site_order(t, seed)
        ts = int(rc["p"] * t)
        s, csize, cln, maxcn, maxcs = O.label_sites(lattice, L, L, 0, order, ts, literal=False)
        perccln = lib.or_span_sites(L, L, s, csize, cln, L)
        if perccln <= 0:
            return None
        canon = canon_from_sites(s)
        b1, b2 = O.bond_list(lattice, L, L, 0)
        nb = len(b1)
        gval = O.f64(nb)
        lib.or_bond_values(1, nb, b1, b2, O.i32(nb), s, perccln, 1.0, 1e-12, gval)
        info = dict(occupied=ts, cln=cln, maxcs=maxcs, perccln=perccln,
                    perccls=int(csize[perccln]), span_sites=int(np.sum(s == perccln)))
        sysin = dict(b1=b1, b2=b2, gval=gval, rhs_rule=0, cur_rule=1, cur_thresh=0.0)
    info["canon_sha256"] = canon_hash(canon)
    info["nclusters"] = int(len(np.unique(canon[canon > 0])))
    return info, sysin


def find_seed(rc, kmax=64):
    O = _oracle()
    if "sseed" in rc or "seed" in rc:  # fixed seeds (the mixed cases)
        r = label_case(rc, 0)
        if r is None:
            raise RuntimeError("no spanning cluster")
        return 0, 0, r
    seeds = O.i32(kmax)
    O.lib().or_trial_seeds(MASTER, kmax, seeds)
    if "ii" in rc:  # a fixed realisation (must span)
        r = label_case(rc, int(seeds[rc["ii"] - 1]))
        if r is None:
            raise RuntimeError("realisation %d does not span" % rc["ii"])
        return rc["ii"], int(seeds[rc["ii"] - 1]), r
    for ii in range(1, kmax + 1):
        r = label_case(rc, int(seeds[ii - 1]))
        if r is not None:
            return ii, int(seeds[ii - 1]), r
    raise RuntimeError("no spanning realisation in %d trials" % kmax)


def solve(args):
    case, tol = args
    rc = CASES[case]
    O = _oracle()
    ii, seed, (info, sysin) = find_seed(rc)
    L = rc["L"]
    t0 = time.time()
    r = O.conductance(rc["lattice"], L, L, 0, sysin["b1"], sysin["b2"], sysin["gval"], itol=2,
                      tol=tol, itmax=10 ** 6, rhs_rule=sysin["rhs_rule"],
                      cur_rule=sysin["cur_rule"], cur_thresh=sysin["cur_thresh"])
    errs = r["errs"]
    hist = [[int(k + 1), float(errs[k])] for k in range(HIST_EVERY - 1, len(errs), HIST_EVERY)]
    return case, tol, ii, seed, info, dict(
        gtop=r["gtop"], gbot=r["gbot"], iter=r["iter"], err=r["err"], seconds=time.time() - t0,
        err_history=hist)


def decades(case):
    """all of TOLS_DECADES from one threaded run; existing solves must match bitwise"""
    rc = CASES[case]
    O = _oracle()
    ii, seed, (info, sysin) = find_seed(rc)
    L = rc["L"]
    t0 = time.time()
    res, errs = O.conductance_decades(rc["lattice"], L, L, 0, sysin["b1"], sysin["b2"],
                                      sysin["gval"], TOLS_DECADES, rhs_rule=sysin["rhs_rule"],
                                      cur_rule=sysin["cur_rule"], cur_thresh=sysin["cur_thresh"],
                                      threads=int(os.environ.get("GOLDEN_THREADS", 2)))
    secs = time.time() - t0
    path = os.path.join(OUT_LARGE if case in LARGE else OUT, case + ".json")
    doc = json.load(open(path)) if os.path.exists(path) else {}
    if doc:
        assert doc["label"]["canon_sha256"] == info["canon_sha256"], case
    kpre = int(os.environ.get("GOLDEN_PREFIX", "0"))
    if kpre:  # the complete err history of the first kpre iterations (bitwise prefix tests)
        doc["err_prefix"] = [float(e) for e in errs[:kpre]]
    solves = doc.setdefault("solves", {})
    for r in res:
        key = "%g" % r["tol"]
        hist = [[int(k + 1), float(errs[k])] for k in range(HIST_EVERY - 1, r["iter"], HIST_EVERY)]
        new = dict(gtop=r["gtop"], gbot=r["gbot"], iter=r["iter"], err=r["err"],
                   true_res=r["true_res"], err_history=hist)
        if key in solves:  # made by the literal linbcg: must be bitwise the same
            old = solves[key]
            for k in ("gtop", "gbot", "iter", "err", "err_history"):
                assert old[k] == new[k], (case, key, k, old[k], new[k])
            new["seconds"] = old.get("seconds")
        solves[key] = new
        print("%s tol %g: iter %d Gtop %.17g Gbot %.17g true_res %.3g"
              % (case, r["tol"], r["iter"], r["gtop"], r["gbot"], r["true_res"]), flush=True)
    doc.update(case=case, recipe=dict(rc, master=MASTER, ii=ii, tseed=seed),
               oracle="oracle/perc_oracle.c (literal linbcg / or_linbcg_sym, O(N alpha) replay)",
               label=dict(doc.get("label", {}), **info))
    doc["decades_run"] = dict(seconds=secs, tols=list(TOLS_DECADES),
                              threads=int(os.environ.get("GOLDEN_THREADS", 2)))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)


def assoc(case, order=1):
    """--assoc: the same solver with its dot products summed in descending
    order (or_linbcg_sym dot_order 1), to the fixture's decades: how far the
    reference solver's own converged Gtop / Gbot move when only the order of
    its sums changes (the floor under any re-associated solve, the GPU's
    included).  Stored as doc["assoc_desc"][tol]; --assoc-tree: pairwise
    (tree) sums, dot_order 2, the association family of a GPU reduction,
    stored as doc["assoc_tree"][tol]."""
    rc = CASES[case]
    O = _oracle()
    ii, seed, (info, sysin) = find_seed(rc)
    L = rc["L"]
    path = os.path.join(OUT, case + ".json")
    doc = json.load(open(path))
    assert doc["label"]["canon_sha256"] == info["canon_sha256"], case
    # every decade of the fixture, the reference tolerance 1e-8 included (round 4);
    # GOLDEN_ASSOC_MIN stops the run early (e.g. 1e-8: only the reference tolerance)
    tmin = float(os.environ.get("GOLDEN_ASSOC_MIN", "0"))
    tols = sorted((float(t) for t in doc["solves"] if float(t) >= tmin), reverse=True)
    t0 = time.time()
    res, _ = O.conductance_decades(rc["lattice"], L, L, 0, sysin["b1"], sysin["b2"], sysin["gval"],
                                   tols, rhs_rule=sysin["rhs_rule"], cur_rule=sysin["cur_rule"],
                                   cur_thresh=sysin["cur_thresh"],
                                   threads=int(os.environ.get("GOLDEN_THREADS", 2)),
                                   dot_order=order)
    key = ASSOC_KEYS[order]
    doc = json.load(open(path))  # re-read: another --assoc run may have written meanwhile
    old = doc.get(key, {})
    new = {"%g" % r["tol"]: dict(gtop=r["gtop"], gbot=r["gbot"], iter=r["iter"],
                                 err=r["err"]) for r in res}
    for k, v in new.items():  # the same run again: bitwise the decades already stored
        if k in old:
            assert old[k] == v, (case, key, k, old[k], v)
    doc[key] = dict(sorted(dict(old, **new).items(), key=lambda kv: -float(kv[0])))
    doc[key + "_seconds"] = max(time.time() - t0, doc.get(key + "_seconds") or 0.0)
    for r in res:
        ref = doc["solves"]["%g" % r["tol"]]
        print("%s %s tol %g: iter %d (asc %d) Gtop %.3e Gbot %.3e rel to asc" % (
            case, key, r["tol"], r["iter"], ref["iter"], abs(r["gtop"] - ref["gtop"]) / ref["gtop"],
            abs(r["gbot"] - ref["gbot"]) / ref["gbot"]), flush=True)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)


def main(cases):
    os.makedirs(OUT, exist_ok=True)
    def done(c, tol):
        path = os.path.join(OUT, c + ".json")
        return os.path.exists(path) and ("%g" % tol) in json.load(open(path)).get("solves", {})
    jobs = [(c, tol) for c in cases for tol in TOLS if not done(c, tol)]
    if not jobs:
        return
    with Pool(min(len(jobs), int(os.environ.get("GOLDEN_PROCS", 6)))) as pool:
        for case, tol, ii, seed, info, res in pool.imap_unordered(solve, jobs):
            path = os.path.join(OUT, case + ".json")
            doc = json.load(open(path)) if os.path.exists(path) else {}
            rc = CASES[case]
            doc.update(case=case, recipe=dict(rc, master=MASTER, ii=ii, tseed=seed),
                       oracle="oracle/perc_oracle.c (literal linbcg, O(N alpha) replay)",
                       label=info)
            doc.setdefault("solves", {})["%g" % tol] = res
            with open(path, "w") as f:
                json.dump(doc, f, indent=1)
            print("%s tol %g: iter %d Gtop %.17g Gbot %.17g (%.0f s)"
                  % (case, tol, res["iter"], res["gtop"], res["gbot"], res["seconds"]),
                  flush=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--decades":
        for c in args[1:] or list(CASES):
            decades(c)
    elif args and args[0] in ASSOC_FLAGS:
        for c in args[1:] or list(CASES):
            assoc(c, ASSOC_FLAGS[args[0]])
    else:
        main(args or list(CASES))
