#!/usr/bin/env python3
"""Timeline of the labeling calls from a rocprofv3 kernel + memory-copy trace
(tools/gpu/label_timeline.sh): per realisation, every dispatch / copy of
perc_occupy_random and perc_label with its start relative to the first and
its duration, and the gaps between them (us).

  python tools/label_timeline.py <dir with *_kernel_trace.csv> [realisation index]
"""
import csv
import glob
import sys


def main(d, which=3):
    ev = []
    for f in glob.glob(d + "/**/*_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    for f in glob.glob(d + "/**/*_memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
    ev.sort()
    # realisations start at k_select_window
    starts = [i for i, e in enumerate(ev) if "k_select_window" in e[2]]
    i0 = starts[which]
    i1 = starts[which + 1] if which + 1 < len(starts) else len(ev)
    t0, prev = ev[i0][0], ev[i0][0]
    for s, e, n in ev[i0:i1]:
        print("%8.1f  gap %6.1f  dur %7.1f  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, n))
        prev = e
    print("span %.1f us" % ((ev[i1 - 1][1] - t0) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
