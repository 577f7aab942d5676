#!/usr/bin/env python3
"""Per-phase times of the resident loop from a PERC_RES_TRACE CSV (wall
clock at 100 MHz): t0 loop top, t1 halo + p(k) in LDS, t2 q and q.p block
sum, t3 after the q.p all-gather, t4 r update + z.r/r.r block sum, t5
after the second all-gather; t0 of the next iteration closes it."""
import sys

import numpy as np


def main(path):
    rows, head = [], None
    for line in open(path):
        if line.startswith("#"):
            head = line.strip()
            continue
        if line.startswith("wg"):
            continue
        rows.append([int(v) for v in line.split(",")])
    a = np.array(rows, dtype=np.float64)
    print(head)
    names = ["halo+p", "q+dot", "gather1", "r upd", "gather2", "to next"]
    for wg in np.unique(a[:, 0]):
        b = a[a[:, 0] == wg]
        b = b[8:-1]  # skip the first iterations (warm-up) and the last
        t = b[:, 2:8]
        nxt = np.roll(b[:, 2], -1)[:-1]
        d = np.diff(t, axis=1)[:-1] * 10.0  # ns
        tail = (nxt - t[:-1, 5]) * 10.0
        per = (nxt - t[:-1, 0]) * 10.0
        cols = [np.median(d[:, i]) for i in range(5)] + [np.median(tail)]
        print("wg %5d: " % wg + "  ".join("%s %.2f us" % (n, c / 1e3) for n, c in zip(names, cols))
              + "  | iteration %.2f us (median), %.2f (mean)" % (np.median(per) / 1e3, per.mean() / 1e3))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
