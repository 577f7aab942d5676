#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd .db or the CSV
kernel_stats) into profiles/<name>.csv: name, calls, total_us, avg_us, pct."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels"))
    # durations are ns in rocpd
    return [(n, int(k), t / 1e3, a / 1e3, p) for n, k, t, a, p in rows]


def short(name):
    n = name.split("(")[0]
    return n.replace("perc::(anonymous namespace)::", "").replace("perc::", "")[:80]


def main(src, dst):
    dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
    rows = from_db(dbs[0])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for n, k, t, a, p in rows:
            w.writerow([short(n), k, "%.1f" % t, "%.3f" % a, "%.3f" % p])
    for n, k, t, a, p in rows[:8]:
        print("%-60s %8d %12.1f us  avg %9.3f us  %6.2f%%" % (short(n), k, t, a, p))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
