#!/usr/bin/env python3
"""The kernel-trace summary of a rocprofv3 database (`<name>_results.db`,
the rocpd SQLite format this ROCm writes by default) as the CSV of
`rocprofv3 --stats --output-format csv` (kernel_stats.csv columns): name,
calls, total / average / min / max duration in ns, percentage of the total.

  python tools/rocpd_stats.py gpurun_out/r5f_prof/bench_results.db > profiles/r5_5_rocprof_stats_L4096.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, lo, hi in rows:
        w.writerow([name, n, tot, round(avg, 3), round(100.0 * tot / total, 4), lo, hi])


if __name__ == "__main__":
    main(sys.argv[1])
