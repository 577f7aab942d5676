#!/usr/bin/env python3
"""Reconcile the PMC passes of tools/pmc_r2.sh with the algorithmic bytes.

For every pass directory (rocprofv3 -f csv output) and each kernel of
interest, take the LAST n dispatches (the same dispatch set in every pass:
tools/pmc_probe.py's fixed work launches) and average each counter.  Read
bytes are computed from the request-size counters (32 / 64 / 128-B EA read
requests: exact, no FETCH_SIZE halving question), write bytes from
WRITE_SIZE; the STREAM copy (512 MB read + 512 MB written per dispatch)
calibrates both.

  python tools/pmc_reconcile.py OUT.csv --last "k_cg_march<1=64" k_copy=16 \
      --algo "k_cg_march<1=R:W" k_copy=R:W  DIR [DIR ...]
  (kernels are named with their first template argument)
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name):
    n = name.replace("perc::(anonymous namespace)::", "").replace("perc::", "")
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\(.*", "", n)


def load(d):
    """kernel base name -> counter -> [per-dispatch value, in dispatch order]"""
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = defaultdict(lambda: defaultdict(list))
    if not path:
        return out
    rows = list(csv.DictReader(open(path[0])))
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
    for r in rows:
        # kernel + first template argument (k_cg_march<1: the q-free P, <2: its B)
        k = short(r["Kernel_Name"]).split(",")[0].rstrip(">")
        out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--last", nargs="+", default=[])
    ap.add_argument("--algo", nargs="+", default=[])
    a = ap.parse_args()
    last = {k: int(v) for k, v in (x.split("=") for x in a.last)}
    algo = {k: tuple(float(t) for t in v.split(":")) for k, v in (x.split("=") for x in a.algo)}
    ctr = defaultdict(dict)  # kernel -> counter -> mean over its last n dispatches
    nd = defaultdict(dict)
    for d in a.dirs:
        for k, cs in load(d).items():
            if k not in last:
                continue
            for c, v in cs.items():
                v = v[-last[k]:]
                ctr[k][c] = sum(v) / len(v)
                nd[k][c] = len(v)
    rows = []
    for k in last:
        if k not in ctr:  # not launched in this probe (another march mode)
            continue
        c = ctr[k]
        rd = None
        if "TCC_EA0_RDREQ_128B_sum" in c:
            rd = (128 * c["TCC_EA0_RDREQ_128B_sum"] + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0)
                  + 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0))
        wr = 1024 * c["WRITE_SIZE"] if "WRITE_SIZE" in c else None
        fetch = 1024 * c["FETCH_SIZE"] if "FETCH_SIZE" in c else None
        ar, aw = algo.get(k, (None, None))
        hit = None
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            hit = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1)
        rows.append(dict(
            kernel=k, dispatches=max(nd[k].values()) if nd.get(k) else 0,
            read_bytes=rd, fetch_size_bytes=fetch, write_bytes=wr,
            algo_read=ar, algo_write=aw,
            read_over_algo=rd / ar if rd and ar else None,
            write_over_algo=wr / aw if wr and aw else None,
            req32=c.get("TCC_EA0_RDREQ_32B_sum"), req64=c.get("TCC_EA0_RDREQ_64B_sum"),
            req128=c.get("TCC_EA0_RDREQ_128B_sum"), rdreq=c.get("TCC_EA0_RDREQ_sum"),
            rdreq_dram=c.get("TCC_EA0_RDREQ_DRAM_sum"), wrreq_dram=c.get("TCC_EA0_WRREQ_DRAM_sum"),
            wrreq=c.get("TCC_EA0_WRREQ_sum"), l2_hit=hit))
    with open(a.out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        for r in rows:
            w.writerow({k: ("%.6g" % v if isinstance(v, float) else v) for k, v in r.items()})
    for r in rows:
        print(" ".join("%s=%s" % (k, ("%.4g" % v if isinstance(v, float) else v))
                       for k, v in r.items()))


if __name__ == "__main__":
    main()
