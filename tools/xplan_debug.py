"""Diagnostic: one sharded tick of test_sharded_churn's shape (world 2) with the xplan
form on and off: compares the summed exchange (c bytes per position) after phase 1 and
the merged outputs.  python tools/xplan_debug.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402,F401

from faasbal import synth  # noqa: E402
from faasbal.sharded import ShardedBalancer  # noqa: E402

st = synth.zipf_state(W=65536, seed=3)
ticks = synth.churn_ticks(st, n_ticks=1, seed=2, tasks_per_tick=65536, join_frac=0.001, expire_frac=0.001,
                          results_per_tick=8192)
tk = ticks[0]
E = len(tk["ev_kind"])
seq = np.full(E, -1, np.int64)
world = 2
outs = {}
for mode in (0, 1):
    bals = [ShardedBalancer(r, world, 65536, len(st["log"]) + 3 * 65536 + 200_000, max_events=20000)
            for r in range(world)]
    for b in bals:
        b.load(st)
        b.set_path("xplan", mode)
    for b in bals:
        b.launch(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, tk["n_new"])
        b.sync()
    ex = [b.exchange().clone() for b in bals]
    tot = ex[0].clone()
    for x in ex[1:]:
        tot += x
    for b in bals:
        b.exchange().copy_(tot)
    torch.cuda.synchronize()
    res = []
    for b in bals:
        b.cont()
        res.append(b.wait())
    tasks = [b.local_assignments() for b in bals]
    outs[mode] = (tot.cpu().numpy(), res, tasks)
    print("mode %d: exchange %d B, results %s" % (mode, tot.numel(), [dict((k, r[k]) for k in ("n_assigned", "n_orphans", "queue_len", "fill_level", "max_free")) for r in res]))
    for r, (tsk, slot) in enumerate(tasks):
        d = np.diff(tsk)
        print("  rank %d: %d local tasks, ascending %s, first bad %s" % (r, len(tsk), bool(np.all(d > 0)),
                                                                     np.nonzero(d <= 0)[0][:5]))
    for b in bals:
        b.close()
# c bytes: mode 0's exchange holds rows after c8, mode 1's not; compare the c8 region by locating it
a0, a1 = outs[0][0], outs[1][0]
print("exchange sizes", len(a0), len(a1))
t0 = np.concatenate([t for t, _ in outs[0][2]])
t1 = np.concatenate([t for t, _ in outs[1][2]])
s0 = np.concatenate([s for _, s in outs[0][2]])
s1 = np.concatenate([s for _, s in outs[1][2]])
o0, o1 = np.argsort(t0), np.argsort(t1)
print("tasks equal:", np.array_equal(t0[o0], t1[o1]), "slots equal:", np.array_equal(s0[o0], s1[o1]))
if len(t0) == len(t1):
    bad = np.nonzero(s0[o0] != s1[o1])[0]
    print("first differing tasks", t0[o0][bad[:10]], s0[o0][bad[:10]], s1[o1][bad[:10]])
n = min(len(a0), len(a1))
diff = np.nonzero(a0[:n] != a1[:n])[0]
print("exchange bytes differing (common prefix):", len(diff), diff[:20])
