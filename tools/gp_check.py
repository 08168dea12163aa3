"""Diagnostic (stamps build): the first configs[4] stream tick with k_plan2 AND the gp
prologue; per queue block k_emit2's round-0 prefix beside k_plan2's."""
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
g = GpuBalancer(W, len(st["log"]) + 8 * T, max_events=E,
                lib_path=os.path.join(REPO, "distributed-faas_amd", "faasbal", "libfaasbal_stamps.so"))
g.set_path("gpcheck", 1)
g.load(st)
tk = ticks[0]
g.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], tk["n_new"], commit=False)
d = g.debug_read().reshape(-1, 16).astype(np.int64)
nbw, nbf = -(-W // 256), -(-len(st["log"]) // 2048)
Qlog = len(st["queue"]) + 2 * len(tk["ev_kind"])
nbq = -(-Qlog // 256)
base = 3 * (nbw + nbf + nbq) + 1024
rows = d[base:base + nbq]
ok = rows[:, 0] > 0
print("nbq %d, rows stamped %d, gshift %s" % (nbq, ok.sum(), set(rows[ok, 5].tolist())))
bad = ok & (rows[:, 1] != rows[:, 2])
print("blocks whose prefix differs from k_plan2's:", bad.sum())
for r in rows[bad][:20]:
    print("  block %d group %d: gp %d plan2 %d (diff %d)" % (r[0] - 1, r[3], r[1], r[2], r[1] - r[2]))
