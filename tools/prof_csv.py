#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (-f csv) per kernel.

  prof_csv.py trace <dir> <out.csv>   kernel_trace.csv -> calls, avg/total us,
                                      and the average over launches that did
                                      work (> 20% of the median: the CG
                                      kernels return at once after the stop
                                      flag, those no-op tails are excluded)
  prof_csv.py pmc <dir> <out.csv>     counter_collection.csv -> per-dispatch
                                      mean of each counter over dispatches
                                      that did work; FETCH_SIZE (kB)
                                      also doubled (gfx950: FETCH_SIZE counts
                                      128-B requests at 64 B,
                                      MI355X_MICROARCH.md § HBM) and in bytes
"""
import csv
import glob
import os
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    n = name.replace("perc::(anonymous namespace)::", "").replace("perc::", "")
    if n.startswith("void rocprim") or "rocprim" in n[:40]:
        return "rocprim::scan"
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:60]


def find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not hits:
        sys.exit("no %s under %s" % (pat, d))
    return hits[0]


def trace(d, out):
    dur = defaultdict(list)
    with open(find(d, "*kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for k, v in dur.items():
        med = statistics.median(v)
        work = [x for x in v if x > 0.2 * med]
        rows.append((k, len(v), sum(v) / 1e3, sum(v) / len(v) / 1e3, len(work),
                     sum(work) / max(len(work), 1) / 1e3))
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "work_calls", "work_avg_us",
                    "percent"])
        for r in rows:
            w.writerow([r[0], r[1], "%.1f" % r[2], "%.3f" % r[3], r[4], "%.3f" % r[5],
                        "%.2f" % (100 * r[2] / tot)])
    for r in rows[:12]:
        print("%-40s %7d calls %12.1f us  avg %9.3f  work %7d avg %9.3f us" % r)


def pmc(d, out):
    vals = defaultdict(lambda: defaultdict(list))
    with open(find(d, "*counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "counter", "dispatches", "mean_per_dispatch", "bytes_per_dispatch",
                    "note"])
        for k, cs in sorted(vals.items()):
            for c, v in sorted(cs.items()):
                # CG launches after the stop flag return at once (zero
                # traffic): average over the dispatches that did work
                top = max(v)
                v = [x for x in v if x > 0.01 * top] or v
                m = sum(v) / len(v)
                if c == "FETCH_SIZE":
                    b, note = m * 1024 * 2, "kB; bytes = 2 x kB x 1024 (gfx950 correction)"
                elif c == "WRITE_SIZE":
                    b, note = m * 1024, "kB; bytes = kB x 1024"
                else:
                    b, note = "", ""
                w.writerow([k, c, len(v), "%.1f" % m, "%.0f" % b if b != "" else "", note])
                print("%-40s %-12s n=%6d mean %14.1f  bytes %s" % (k, c, len(v), m,
                                                                 "%.4g" % b if b != "" else "-"))


if __name__ == "__main__":
    {"trace": trace, "pmc": pmc}[sys.argv[1]](sys.argv[2], sys.argv[3])
