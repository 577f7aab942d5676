#!/usr/bin/env python3
"""Summarise a PERC_MARCH_TRACE csv (per-wave wall-clock stamps of the march
P / B launches, 100 MHz): launch span, entry ramp, walk durations, exit
tail, per-XCC means.  python tools/march_trace_summary.py trace.csv"""
import sys

import numpy as np


def main(path):
    rows = []
    for line in open(path):
        if line.startswith("#") or line.startswith("iter"):
            continue
        it, k, w, t0, t1, t2, xcc, hw = line.strip().split(",")
        rows.append((int(it), k, int(w), int(t0), int(t1), int(t2), int(xcc), int(hw)))
    a = np.array([(r[0], r[1] == "B", r[2], r[3], r[4], r[5], r[6], r[7]) for r in rows],
                 dtype=np.int64)
    for it in np.unique(a[:, 0]):
        for kb in (0, 1):
            s = a[(a[:, 0] == it) & (a[:, 1] == kb) & (a[:, 3] > 0)]
            if len(s) == 0:
                continue
            t0, t1, t2, xcc = s[:, 3] * 0.01, s[:, 4] * 0.01, s[:, 5] * 0.01, s[:, 6]  # us
            base = t0.min()
            walk = t1 - t0
            q = lambda v, p: np.percentile(v, p)
            print("iter %d %s: waves %d span %.1f us | entry +%.1f p50 +%.1f max | walk p5 %.1f p50 %.1f "
                  "p95 %.1f max %.1f | walk end p50 +%.1f p95 +%.1f max +%.1f | exit max +%.1f"
                  % (it, "B" if kb else "P", len(s), t2.max() - base, q(t0 - base, 50),
                     (t0 - base).max(), q(walk, 5), q(walk, 50), q(walk, 95), walk.max(),
                     q(t1 - base, 50), q(t1 - base, 95), (t1 - base).max(), (t2 - base).max()))
            per = ["%d:%.1f" % (x, walk[xcc == x].mean()) for x in np.unique(xcc)]
            print("   walk mean per XCC: " + " ".join(per))
            nw = len(s)
            strips = 32
            wi = s[:, 2]
            strip = wi % strips
            edge = (strip == 0) | (strip == strips - 1)
            hw = s[:, 7]
            # gfx9 HW_ID: wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13, tg 19:16
            fields = dict(wave_slot=hw & 15, simd=(hw >> 4) & 3, cu=(hw >> 8) & 15, se=(hw >> 13) & 7,
                          tg=(hw >> 16) & 15, wave_in_wg=s[:, 2] % 4,
                          band_parity=(s[:, 2] // 32) % 2)
            for name, f in fields.items():
                vals = np.unique(f)
                if len(vals) > 1 and len(vals) <= 16:
                    print("   walk mean by %s: %s" % (name, " ".join(
                        "%d:%.1f" % (v, walk[f == v].mean()) for v in vals)))
            # entry order on a CU (rank of t_entry among the waves of the same cu/se/xcc)
            key = xcc * 4096 + ((hw >> 8) & 15) * 16 + ((hw >> 13) & 7)
            order = np.zeros(len(s), np.int64)
            for kk in np.unique(key):
                idx = np.nonzero(key == kk)[0]
                order[idx[np.argsort(t0[idx], kind="stable")]] = np.arange(len(idx))
            print("   walk mean by entry rank on its CU: %s" % " ".join(
                "%d:%.1f" % (v, walk[order == v].mean()) for v in np.unique(order)[:16]))
            print("   walk mean edge strips %.1f interior %.1f; slowest 1%% waves: strips %s"
                  % (walk[edge].mean(), walk[~edge].mean(),
                     np.bincount(strip[walk >= q(walk, 99)], minlength=strips).nonzero()[0][:12]))


if __name__ == "__main__":
    main(sys.argv[1])
