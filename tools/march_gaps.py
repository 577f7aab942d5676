#!/usr/bin/env python3
"""Dispatch gaps between consecutive march launches from a rocprofv3 kernel
trace (tools/gpu/march_gaps.sh): start of each P / B launch minus the end of
the launch before it, percentiles (us), and the launches' own durations.

  python tools/march_gaps.py <dir with *_kernel_trace.csv>
"""
import csv
import glob
import sys

import numpy as np


def main(d):
    ev = []
    for f in glob.glob(d + "/**/*_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    gaps = {"P->B": [], "B->P": []}
    dur = {"P": [], "B": []}
    for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
        k0 = "P" if "k_cg_march<1," in n0 else ("B" if "k_cg_march<2," in n0 else None)
        k1 = "P" if "k_cg_march<1," in n1 else ("B" if "k_cg_march<2," in n1 else None)
        if k0 and k1 and k0 != k1:
            gaps[k0 + "->" + k1].append((s1 - e0) / 1e3)
        if k0:
            dur[k0].append((e0 - s0) / 1e3)
    for k, v in list(gaps.items()) + list(dur.items()):
        v = np.array(v)
        if len(v):
            print("%-5s n %6d  p5 %7.2f  p50 %7.2f  p95 %7.2f  mean %7.2f us" % (
                k, len(v), np.percentile(v, 5), np.percentile(v, 50), np.percentile(v, 95), v.mean()))


if __name__ == "__main__":
    main(sys.argv[1])
