"""Probe: host-side time split of a committed streaming tick (configs[4] per GPU):
fb_tick_launch (validation + staging + H2D + enqueue), fb_tick_wait, fb_tick_commit."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
import numpy as np
from faasbal import GpuBalancer, synth

W, T, K = 1 << 20, 65536, 30
st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
ticks = synth.stream_ticks(st, n_ticks=K + 5, seed=2, tasks_per_tick=T, results_per_tick=T)
g = GpuBalancer(W, len(st["log"]) + (K + 8) * 2 * T, max_events=max(len(t["ev_kind"]) for t in ticks), device=0)
g.load(st)
carried = 0
acc = np.zeros(4)
for i, tk in enumerate(ticks):
    n = carried + tk["n_new"]
    t0 = time.perf_counter()
    g.launch(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
    t1 = time.perf_counter()
    r = g.wait()
    t2 = time.perf_counter()
    g.commit()
    g.sync()
    t3 = time.perf_counter()
    carried = n + r["n_orphans"] - r["n_assigned"]
    if i >= 5:
        acc += [t1 - t0, t2 - t1, t3 - t2, t3 - t0]
acc /= K
print("per tick us: launch %.1f  wait %.1f  commit %.1f  total %.1f" % tuple(acc * 1e6))
