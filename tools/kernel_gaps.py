"""Per-tick device timeline from a rocprofv3 --kernel-trace directory alone: for the
ticks anchored at ANCHOR (default k_ev_link), the median start, duration and idle gap
before each kernel of the modal per-tick sequence, and the median tick period.
Usage: kernel_gaps.py TRACE_DIR [ANCHOR]"""
import csv
import glob
import os
import sys
from collections import Counter

import numpy as np


def short(n):
    return n.split("(")[0].replace("void ", "").replace("fb::", "").split("<")[0]


def main(d, anchor="k_ev_link"):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(p)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    idx = [i for i, k in enumerate(ks) if k[0] == anchor]
    ticks = [ks[a:b] for a, b in zip(idx, idx[1:])]
    seqs = Counter(tuple(k[0] for k in t) for t in ticks)
    modal, n = seqs.most_common(1)[0]
    sel = [t for t in ticks if tuple(k[0] for k in t) == modal]
    print("ticks %d, modal sequence %d of them" % (len(ticks), n))
    print("%-16s %9s %9s %9s" % ("kernel", "start", "dur", "gap"))
    for j, name in enumerate(modal):
        st = np.median([(t[j][1] - t[0][1]) / 1e3 for t in sel])
        du = np.median([(t[j][2] - t[j][1]) / 1e3 for t in sel])
        gp = np.median([((t[j][1] - t[j - 1][2]) if j else 0) / 1e3 for t in sel])
        print("%-16s %9.1f %9.1f %9.1f" % (name, st, du, gp))
    per = [(b[0][1] - a[0][1]) / 1e3 for a, b in zip(ticks, ticks[1:])]
    busy = np.median([sum(k[2] - k[1] for k in t) / 1e3 for t in sel])
    tail = np.median([(b[0][1] - a[-1][2]) / 1e3 for a, b in zip(ticks, ticks[1:]) if a in sel])
    print("tick period median %.1f us; busy %.1f us; gap from the tick's last kernel to the next tick's first %.1f us"
          % (np.median(per), busy, tail))


if __name__ == "__main__":
    main(*sys.argv[1:])
