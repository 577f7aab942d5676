#!/usr/bin/env python3
"""Generate golden fixtures from the compiled reference (oracle/_ref).

TEST INFRASTRUCTURE.  Runs each reference binary built by
oracle/build_ref.sh (flang -O2 from /root/reference/Fortran sources, with the
real libgfortran rand/srand) in a scratch directory, then stores

  * its formatted output files (bond.txt, site.txt, ...) gzipped, byte-exact;
  * md5 of the verbose debug logs (bondocc.txt, siteocc.txt, sbdebug.txt);
  * scalars parsed from stdout (largest / spanning cluster, per-iteration
    linbcg err, Conductance Gtop Gbot, Vint where the variant prints it)

under tests/golden/<variant>/.  Only data is committed: no reference source.

Usage: python tests/golden/make_golden.py   (needs oracle/_ref built here)
"""
import gzip
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_BIN = os.path.join(REPO, "oracle", "_ref")

# variant -> (program kind, parameters as edited by oracle/build_ref.sh)
VARIANTS = {
    "sq_bondc_p50": ("bondc", dict(lattice=0, m=50, n=50, pbc=0, pb=0.50, seed=626504)),
    "sq_bondc_p60": ("bondc", dict(lattice=0, m=50, n=50, pbc=0, pb=0.60, seed=626504)),
    "sq_bondc_p60_tight": ("bondc", dict(lattice=0, m=50, n=50, pbc=0, pb=0.60, seed=626504,
                                         tol=1e-14, itmax=200000)),
    "sq_bondc_p60_pbc": ("bondc", dict(lattice=0, m=50, n=50, pbc=1, pb=0.60, seed=626504)),
    "sq_bondc_20x30_p55": ("bondc", dict(lattice=0, m=20, n=30, pbc=0, pb=0.55, seed=777)),
    "tri_bondc_p35": ("bondc", dict(lattice=1, m=50, n=50, pbc=0, pb=0.35, seed=62703)),
    "tri_bondc_p35_tight": ("bondc", dict(lattice=1, m=50, n=50, pbc=0, pb=0.35, seed=62703,
                                          tol=1e-14, itmax=200000)),
    "tri_bondc_p40_pbc": ("bondc", dict(lattice=1, m=50, n=50, pbc=1, pb=0.40, seed=62703)),
    "sq_site": ("site", dict(lattice=0, m=50, n=50, pbc=0, ps=0.60, seed=1080115)),
    "sq_site_64": ("site", dict(lattice=0, m=64, n=64, pbc=0, ps=0.60, seed=1080115)),
    "sq_site_pbc": ("site", dict(lattice=0, m=50, n=50, pbc=1, ps=0.60, seed=1080115)),
    "tri_site": ("site", dict(lattice=1, m=50, n=50, pbc=0, ps=0.548, seed=143285)),
    "sq_sitebond": ("sitebond", dict(lattice=0, m=50, n=50, pbc=0, ps=0.50, pb=0.50,
                                     sseed=143285, bseed=43716)),
    "sq_sitebond_p9": ("sitebond", dict(lattice=0, m=50, n=50, pbc=0, ps=0.90, pb=0.60,
                                        sseed=143285, bseed=43716)),
    "tri_sitebond": ("sitebond", dict(lattice=1, m=10, n=10, pbc=0, ps=0.50, pb=0.50,
                                      sseed=143285, bseed=43716)),
    # bonds first, then sites (Square/bondsite.f, Triangular/bondsite.f)
    "sq_bondsite": ("bondsite", dict(lattice=0, m=10, n=10, pbc=0, ps=0.50, pb=0.50,
                                     sseed=143285, bseed=43716)),
    "sq_bondsite_30": ("bondsite", dict(lattice=0, m=30, n=30, pbc=0, ps=0.80, pb=0.70,
                                        sseed=143285, bseed=43716)),
    "sq_bondsite_30_pbc": ("bondsite", dict(lattice=0, m=30, n=30, pbc=1, ps=0.80, pb=0.70,
                                            sseed=143285, bseed=43716)),
    "tri_bondsite": ("bondsite", dict(lattice=1, m=10, n=10, pbc=0, ps=0.50, pb=0.50,
                                      sseed=143285, bseed=43716)),
    "tri_bondsite_30": ("bondsite", dict(lattice=1, m=30, n=30, pbc=0, ps=0.70, pb=0.60,
                                         sseed=143285, bseed=43716)),
    "sq_bond_cond": ("bond_cond", dict(lattice=0, m=10, n=10, pbc=0, numtrials=1, seed=58302)),
    "sq_bond_cond_3t": ("bond_cond", dict(lattice=0, m=12, n=12, pbc=0, numtrials=3,
                                          seed=58302)),
    "tri_bond_cond": ("bond_cond", dict(lattice=1, m=10, n=10, pbc=0, numtrials=1, seed=58302)),
    # threshold scans (Square/bond_perc.f, site_perc.f): per trial tseed, first
    # spanning fraction, largest and spanning cluster sizes
    "sq_bond_perc": ("bond_perc", dict(lattice=0, m=50, n=50, pbc=0, numtrials=10, seed=58302)),
    "sq_bond_perc_pbc": ("bond_perc", dict(lattice=0, m=40, n=30, pbc=1, numtrials=10,
                                           seed=58302)),
    "tri_bond_perc": ("bond_perc", dict(lattice=1, m=50, n=50, pbc=0, numtrials=10, seed=58302)),
    "sq_site_perc": ("site_perc", dict(lattice=0, m=50, n=50, pbc=0, numtrials=40, seed=58302)),
    "tri_site_perc": ("site_perc", dict(lattice=1, m=50, n=50, pbc=0, numtrials=40, seed=58302)),
    "sq_site_perc_pbc": ("site_perc", dict(lattice=0, m=36, n=44, pbc=1, numtrials=40,
                                           seed=58302)),
    # mixed threshold scans (Square/sb_perc.f, bs_perc.f): points = the ps
    # (sb) / pb (bs) values as edited in oracle/build_ref.sh, iters per point
    "sq_sb_perc": ("sb_perc", dict(lattice=0, m=50, n=50, pbc=0, seed=8811064, iters=5,
                                   points=[0.65 + 0.10 * i for i in range(4)])),
    "tri_sb_perc": ("sb_perc", dict(lattice=1, m=50, n=50, pbc=0, seed=8811064, iters=5,
                                    points=[0.60 + 0.10 * i for i in range(4)])),
    "sq_bs_perc": ("bs_perc", dict(lattice=0, m=10, n=10, pbc=0, seed=229102, iters=8,
                                   points=[0.55 + 0.10 * i for i in range(5)])),
    "tri_bs_perc": ("bs_perc", dict(lattice=1, m=10, n=10, pbc=0, seed=229102, iters=8,
                                    points=[0.55 + 0.10 * i for i in range(5)])),
}

KEEP = {"bond.txt", "bondorder.txt", "site.txt", "siteorder.txt", "bondlist.txt",
        "sbsite.txt", "sbbond.txt", "bondcond.txt", "bond_perc.txt", "site_perc.txt",
        "sb_perc.txt", "bs_perc.txt", "bssite.txt", "bsbond.txt"}
MD5_ONLY = {"bondocc.txt", "siteocc.txt", "sbdebug.txt", "bsdebug.txt"}
NUM = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[EeDd][-+]?\d+)?"


def fnum(s):
    return float(s.replace("D", "E").replace("d", "e"))


def parse_stdout(text, sitebond_sizes_fix=False):
    meta = {}
    m = re.search(r"largest overall cluster number:\s*(\d+)", text)
    if m:
        meta["maxcn"] = int(m.group(1))
    m = re.search(r"largest overall cluster size:\s*(\d+)", text)
    if m:
        meta["maxcs"] = int(m.group(1))
    m = re.search(r"infinite cluster number:\s*(\d+)", text)
    meta["perccln"] = int(m.group(1)) if m else 0
    m = re.search(r"infinite cluster size:\s*(\d+)", text)
    meta["perccls"] = int(m.group(1)) if m else 0
    errs = [(int(a), fnum(b)) for a, b in
            re.findall(r"iter=\s*(\d+)\s+err=\s*(" + NUM + ")", text)]
    if errs:
        meta["linbcg_err"] = [e for _, e in errs]
        meta["iter"] = errs[-1][0]
    m = re.search(r"Conductance:\s*(" + NUM + r")\s+(" + NUM + ")", text)
    if m:
        meta["gtop"] = fnum(m.group(1))
        meta["gbot"] = fnum(m.group(2))
    # Vint dump (uncommented write in the *_p60 / *_p35 variants) sits between
    # the last ' iter=' line and 'Calculating currents'
    if "Calculating currents" in text and errs:
        tail = text[text.rfind("iter="):text.find("Calculating currents")]
        tail = tail.split("\n", 1)[1] if "\n" in tail else ""
        vals = [fnum(x) for x in re.findall(NUM, tail)]
        if vals:
            meta["vint"] = vals
    return meta


def run_variant(name):
    kind, params = VARIANTS[name]
    exe = os.path.join(REF_BIN, name)
    if not os.path.exists(exe):
        raise SystemExit("missing %s: run oracle/build_ref.sh first" % exe)
    work = tempfile.mkdtemp(prefix="percgold.")
    try:
        proc = subprocess.run([exe], cwd=work, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, timeout=600)
        text = proc.stdout.decode("ascii", "replace")
        meta = {"kind": kind, "params": params}
        meta.update(parse_stdout(text))
        outdir = os.path.join(HERE, name)
        os.makedirs(outdir, exist_ok=True)
        meta["files"] = {}
        for fn in sorted(os.listdir(work)):
            path = os.path.join(work, fn)
            data = open(path, "rb").read()
            md5 = hashlib.md5(data).hexdigest()
            if fn in KEEP:
                with gzip.GzipFile(os.path.join(outdir, fn + ".gz"), "wb",
                                   mtime=0) as g:
                    g.write(data)
                meta["files"][fn] = md5
            elif fn in MD5_ONLY:
                meta["files"][fn] = md5
        with open(os.path.join(outdir, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        return meta
    finally:
        shutil.rmtree(work, ignore_errors=True)


def main(argv):
    names = argv[1:] or sorted(VARIANTS)
    for name in names:
        meta = run_variant(name)
        keys = {k: meta[k] for k in ("perccln", "perccls", "iter", "gtop", "gbot")
                if k in meta}
        print(name, keys, file=sys.stderr)


if __name__ == "__main__":
    main(sys.argv)
