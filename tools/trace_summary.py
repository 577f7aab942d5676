#!/usr/bin/env python3
"""Per-kernel count / average / median (us) from a rocprofv3 -f csv
kernel_trace.csv, sorted by total time.

  python tools/trace_summary.py DIR/run_kernel_trace.csv [--top 25]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        n = r["Kernel_Name"].replace("perc::(anonymous namespace)::", "").replace("void ", "")
        agg[n[:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print("%-70s n=%5d avg=%9.2f med=%9.2f us" % (n, len(v), sum(v) / len(v), sorted(v)[len(v) // 2]))


if __name__ == "__main__":
    main()
