#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd .db) into
profiles/<name>.csv: kernel, calls, total_us, avg_us, percent.
(The rocpd `top_kernels` view reports durations in microseconds.)"""
import csv
import glob
import os
import re
import sqlite3
import sys


def short(name):
    n = name.replace("perc::(anonymous namespace)::", "").replace("perc::", "")
    n = re.sub(r"\(.*", "", n) if not n.startswith("void rocprim") else "rocprim::scan"
    return n[:80]


def main(src, dst):
    db = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels"))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for n, k, t, a, p in rows:
            w.writerow([short(n), k, "%.1f" % t, "%.3f" % a, "%.3f" % p])
    for n, k, t, a, p in rows[:10]:
        print("%-28s %8d %14.1f us  avg %10.3f us  %6.2f%%" % (short(n), k, t, a, p))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
