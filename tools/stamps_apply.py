"""Diagnostic: k_ev_apply_ll's blocks on the streaming tick (libfaasbal_stamps.so): entry
and exit (realtime, 100 MHz) of its message blocks and its slot-purge blocks, relative to
the kernel's first entry, medians over ticks."""
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
                lib_path=os.environ.get("FAASBAL_STAMPS_LIB") or
                os.path.join(REPO, "distributed-faas_amd", "faasbal", "libfaasbal_stamps.so"))
g.load(st)
carried = 0
res = []
for i, tk in enumerate(ticks):
    n = carried + tk["n_new"]
    g.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n_pending=n,
           commit=False, outputs=False)
    r = g.last
    if i >= 5:
        nba, nbw = -(-len(tk["ev_kind"]) // 256), -(-W // 256)
        d = g.debug_read().reshape(-1, 16).astype(np.int64)[: nba + nbw]
        e0 = d[:, 13].min()
        ent, ext = (d[:, 13] - e0) / 100.0, (d[:, 14] - e0) / 100.0
        res.append([np.percentile(ent[:nba], [50, 100]), np.percentile(ext[:nba], [50, 90, 100]),
                    np.percentile(ent[nba:], [50, 100]), np.percentile(ext[nba:], [50, 90, 100])])
    g.commit()
    carried = n + int(r["n_orphans"]) - int(r["n_assigned"])
m = [np.median(np.array([x[k] for x in res]), axis=0) for k in range(4)]
print("k_ev_apply_ll us from the first block entry (medians over %d ticks):" % len(res))
print("  message blocks: entry p50 %.2f max %.2f; exit p50 %.2f p90 %.2f max %.2f" % (*m[0], *m[1]))
print("  purge blocks:   entry p50 %.2f max %.2f; exit p50 %.2f p90 %.2f max %.2f" % (*m[2], *m[3]))
