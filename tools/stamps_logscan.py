"""Diagnostic: k_logscan's phases on the streaming tick (libfaasbal_stamps.so): per block
the bitmap copy (stamp 0 -> 1, shader cycles) and the tile loop (1 -> 15), block entry /
exit offsets (realtime, 100 MHz) relative to the kernel's first entry.  The rows of the
last kernel that stamped are those whose exit lies within 100 us of the newest exit."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
from faasbal import synth  # noqa: E402
from faasbal.balancer import GpuBalancer  # noqa: E402

W, T, K = 1 << 20, 65536, 20
st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
ticks = synth.stream_ticks(st, n_ticks=K + 5, seed=2, tasks_per_tick=T, results_per_tick=T)
E = max(len(t["ev_kind"]) for t in ticks)
g = GpuBalancer(W, len(st["log"]) + (K + 8) * 2 * T, max_events=E,
                lib_path=os.path.join(REPO, "distributed-faas_amd", "faasbal", "libfaasbal_stamps.so"))
g.load(st)
carried = 0
cp, lp, ent, ext, nb = [], [], [], [], []
for i, tk in enumerate(ticks):
    n = carried + tk["n_new"]
    g.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n_pending=n,
           commit=False, outputs=False)
    r = g.last
    if i >= 5:
        d = g.debug_read().reshape(-1, 16).astype(np.int64)
        live = (d[:, 13] > 0) & (d[:, 14] > 0) & (d[:, 1] > 0)
        newest = d[live, 14].max()
        rows = d[live & (d[:, 14] > newest - 10000)]
        cp.append(np.median(rows[:, 1] - rows[:, 0]))
        lp.append(np.median(rows[:, 15] - rows[:, 1]))
        e0 = rows[:, 13].min()
        ent.append(np.percentile(rows[:, 13] - e0, [50, 90, 100]) / 100.0)
        ext.append(np.percentile(rows[:, 14] - e0, [50, 90, 100]) / 100.0)
        nb.append(len(rows))
    g.commit()
    carried = n + int(r["n_orphans"]) - int(r["n_assigned"])
print("k_logscan rows per tick %d; bitmap copy median %d cyc, tile loop median %d cyc"
      % (np.median(nb), np.median(cp), np.median(lp)))
print("entry offset us p50/p90/max", np.median(np.array(ent), axis=0))
print("exit offset us p50/p90/max", np.median(np.array(ext), axis=0))
