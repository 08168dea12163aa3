"""Diagnostic: the first configs[4] stream tick (a general message tick at 1 M workers)
through k_plan2 (gp 0) and without it (gp 1): results and the first differing tasks."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
from faasbal import synth  # noqa: E402
from faasbal.balancer import GpuBalancer  # noqa: E402

W, T = 1 << 20, 65536
st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
ticks = synth.stream_ticks(st, n_ticks=2, seed=2, tasks_per_tick=T, results_per_tick=T)
E = max(len(t["ev_kind"]) for t in ticks)
cap = len(st["log"]) + 8 * T
outs = []
for gp in (0, 1):
    g = GpuBalancer(W, cap, max_events=E)
    g.set_path("gp", gp)
    g.load(st)
    tk = ticks[0]
    a = g.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], tk["n_new"],
               commit=False)
    print("gp", gp, {k: v for k, v in g.last.items()})
    outs.append(a)
    del g
for k in ("assign", "orphans", "evicted", "reconnect"):
    x, y = outs[0][k], outs[1][k]
    if len(x) != len(y):
        print(k, "lengths", len(x), len(y))
        continue
    d = np.nonzero(x != y)[0]
    print(k, "len", len(x), "differ", len(d), "first", d[:10], x[d[:5]] if len(d) else "", y[d[:5]] if len(d) else "")
x, y = outs[0]["assign"], outs[1]["assign"]
inv = {int(s): i for i, s in enumerate(x)}
d = np.nonzero(x != y)[0]
print("gp1 task -> gp0 task of the same slot:", [(int(i), inv.get(int(y[i]), -1)) for i in d[:12]])
print("... around 1000 differing:", [(int(i), inv.get(int(y[i]), -1)) for i in d[1000:1006]])
runs = np.split(d, np.nonzero(np.diff(d) != 1)[0] + 1)
print("differing runs:", len(runs), [(int(r[0]), int(r[-1])) for r in runs[:12]])
