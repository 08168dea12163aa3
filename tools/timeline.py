"""Summarise a rocprofv3 trace directory (kernel / memory-copy / HIP API CSVs) of the
streaming probe into a median per-tick timeline: every device event of the tick in
order with its start relative to the tick's k_ev_link, its duration, the idle gap
before it, and the host call that enqueued it (start relative to the same origin);
then the HIP API time per function and tick.  Usage: timeline.py TRACE_DIR [ANCHOR_KERNEL]"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np


def rows(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def short(n):
    n = n.split("(")[0]
    for p in ("void ", "fb::"):
        n = n.replace(p, "")
    return n[:28]


def main(d, anchor="k_ev_link"):
    ev = []
    for r in rows(d, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Correlation_Id"]))
    for r in rows(d, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")[:12],
                   r.get("Correlation_Id", "")))
    api = rows(d, "*hip_api_trace.csv")
    byc = {r["Correlation_Id"]: r for r in api}
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2].startswith(anchor)]
    if len(starts) < 4:
        print("fewer than 4 ticks in the trace")
        return
    seqs = []
    for a, b in zip(starts[:-1], starts[1:]):
        seqs.append(ev[a:b])
    key = lambda s: tuple(e[2] for e in s)
    cnt = defaultdict(int)
    for s in seqs:
        cnt[key(s)] += 1
    modal = max(cnt, key=cnt.get)
    use = [s for s in seqs if key(s) == modal]
    print("ticks %d, modal sequence %d of them" % (len(seqs), len(use)))
    print("%-30s %9s %9s %9s %10s %10s" % ("event", "start", "dur", "gap", "api_start", "api_dur"))
    n = len(modal)
    st = np.zeros((len(use), n)); du = np.zeros((len(use), n)); gp = np.zeros((len(use), n))
    ast = np.full((len(use), n), np.nan); adu = np.full((len(use), n), np.nan)
    for k, s in enumerate(use):
        t0 = s[0][0]
        prev_end = None
        for j, e in enumerate(s):
            st[k, j] = (e[0] - t0) / 1e3
            du[k, j] = (e[1] - e[0]) / 1e3
            gp[k, j] = 0 if prev_end is None else (e[0] - prev_end) / 1e3
            prev_end = e[1] if prev_end is None else max(prev_end, e[1])
            a = byc.get(e[3])
            if a is not None:
                ast[k, j] = (int(a["Start_Timestamp"]) - t0) / 1e3
                adu[k, j] = (int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3
    for j in range(n):
        print("%-30s %9.1f %9.1f %9.1f %10.1f %10.1f" % (modal[j], np.median(st[:, j]), np.median(du[:, j]),
                                                       np.median(gp[:, j]), np.nanmedian(ast[:, j]) if
                                                       np.isfinite(ast[:, j]).any() else np.nan,
                                                       np.nanmedian(adu[:, j]) if np.isfinite(adu[:, j]).any()
                                                       else np.nan))
    per = [(s[-1][1] - s[0][0]) / 1e3 for s in use]
    nxt = [(ev[starts[i + 1]][0] - ev[starts[i]][0]) / 1e3 for i in range(len(starts) - 1)]
    print("tick period (link to link) median %.1f us; busy (sum of durations) %.1f us"
          % (np.median(nxt), np.median(du.sum(axis=1))))
    # host API time per function between consecutive link starts (median per tick)
    if api:
        lo, hi = ev[starts[len(starts) // 4]][0], ev[starts[-1]][0]
        nt = len([i for i in starts if lo <= ev[i][0] < hi])
        tot = defaultdict(float); num = defaultdict(int)
        for r in api:
            s0 = int(r["Start_Timestamp"])
            if lo <= s0 < hi:
                tot[r["Function"]] += (int(r["End_Timestamp"]) - s0) / 1e3
                num[r["Function"]] += 1
        print("HIP API per tick over %d ticks:" % nt)
        for f in sorted(tot, key=tot.get, reverse=True)[:20]:
            print("  %-36s %8.1f us  %6.1f calls" % (f, tot[f] / nt, num[f] / nt))


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:3])
