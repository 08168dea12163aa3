"""Diagnostic: k_emit_win's phases on the streaming tick (libfaasbal_stamps.so): per chunk
workgroup the classification (stamp 0 -> 1), the look-back chains (1 -> 2) and the
emission (2 -> 15), in shader cycles, and entry / exit offsets (realtime, 100 MHz) from
the kernel's first entry, medians over ticks."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
from faasbal import synth  # noqa: E402
from faasbal.balancer import GpuBalancer  # noqa: E402

ROW0 = 8192
W, T, K = 1 << 20, 65536, 20
st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
ticks = synth.stream_ticks(st, n_ticks=K + 5, seed=2, tasks_per_tick=T, results_per_tick=T)
E = max(len(t["ev_kind"]) for t in ticks)
g = GpuBalancer(W, len(st["log"]) + (K + 8) * 2 * T, max_events=E,
                lib_path=os.path.join(REPO, "distributed-faas_amd", "faasbal", "libfaasbal_stamps.so"))
g.load(st)
carried = 0
res = []
split = []
for i, tk in enumerate(ticks):
    n = carried + tk["n_new"]
    g.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n_pending=n,
           commit=False, outputs=False)
    r = g.last
    if i >= 5:
        d = g.debug_read().reshape(-1, 16).astype(np.int64)[ROW0:ROW0 + 4096]
        newest = d[:, 14].max()
        rows = d[(d[:, 13] > 0) & (d[:, 14] > newest - 10000) & (d[:, 15] > 0)]
        e0 = rows[:, 13].min()
        full = rows[rows[:, 2] > 0]
        res.append([len(rows), np.median(full[:, 1] - full[:, 0]), np.median(full[:, 2] - full[:, 1]),
                    np.percentile(rows[:, 15] - rows[:, 2], 90), np.percentile((rows[:, 13] - e0) / 100.0, 100),
                    np.percentile((rows[:, 14] - e0) / 100.0, 50), np.percentile((rows[:, 14] - e0) / 100.0, 100)])
        nb = -(-len(tk["ev_kind"]) // 1024)  # back chunks come first (chunk = row)
        ix = np.nonzero((d[:, 13] > 0) & (d[:, 14] > newest - 10000) & (d[:, 15] > 0))[0]
        back, rest = rows[ix < nb], rows[ix >= nb]
        fr = rest[rest[:, 4] > 0]
        split.append([np.median(back[:, 4] - back[:, 1]) if len(back) else 0,
                      np.median(fr[:, 4] - fr[:, 1]) if len(fr) else 0,
                      np.median(fr[:, 2] - fr[:, 4]) if len(fr) else 0,
                      (back[:, 14].max() - e0) / 100.0 if len(back) else 0,
                      (rest[:, 14].max() - e0) / 100.0 if len(rest) else 0])
    g.commit()
    carried = n + int(r["n_orphans"]) - int(r["n_assigned"])
m = np.median(np.array(res), axis=0)
print("k_emit_win: %d chunks; classify %d cyc, look-back %d cyc, emission p90 %d cyc (medians); "
      "entry max +%.2f us, exit p50 +%.2f / max +%.2f us" % tuple(m))
if split:
    m2 = np.median(np.array(split), axis=0)
    print("  back chunks: own chain %d cyc, last exit +%.2f us; front / window chunks: own chain %d cyc, "
          "wait for the back total %d cyc, last exit +%.2f us" % (m2[0], m2[3], m2[1], m2[2], m2[4]))
