#!/usr/bin/env python3
"""Little's-law summary of tools/pmc_level.sh: per kernel, cycles per XCD,
mean outstanding EA read / write requests, requests per cycle, mean latency."""
import collections
import csv
import glob
import sys


def load(d, last):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    v = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"].split("<")[0].split("::")[-1].split("(")[0]
        v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(x[-last[k]:]) / last[k] for c, x in cs.items()} for k, cs in v.items() if k in last}


last = {"k_cg_march": 64, "k_cg_b": 64, "k_copy": 16}
for d in sys.argv[1:]:
    a, b = load(d, last), load(d + "_n", last)
    for k in last:
        cyc = a[k]["GRBM_GUI_ACTIVE"] / 8
        rl, wl = a[k]["TCC_EA0_RDREQ_LEVEL_sum"] / cyc, a[k]["TCC_EA0_WRREQ_LEVEL_sum"] / cyc
        rn, wn = b[k]["TCC_EA0_RDREQ_sum"], b[k]["TCC_EA0_WRREQ_sum"]
        print("%-22s %-11s cycles %8.0f  rd outstanding %7.0f (%5.2f req/cyc, latency %5.0f)  "
              "wr outstanding %7.0f (%5.2f req/cyc, latency %5.0f)"
              % (d.split("/")[-1], k, cyc, rl, rn / cyc, rl / (rn / cyc), wl, wn / cyc, wl / (wn / cyc)))
