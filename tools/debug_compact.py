"""Diagnostic: the compact readback path (GpuBalancer.tick(compact=True)) against the
per-task readback on the same functional tick, for the golden vectors' first ticks."""
import glob
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from faasbal import GpuBalancer  # noqa: E402
from oracle import fixture_ticks  # noqa: E402

for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "cfg*.npz"))):
    z = np.load(path)
    W = int(z["W"])
    max_e = max(1, int(np.diff(z["ev_off"]).max(initial=0)))
    g = GpuBalancer(2 * W + max_e, len(z["init_log"]) + len(z["exp_assign"]) + 64, max_events=max_e + 1)
    g.load_state(z["init_reg"], z["init_free"], z["init_hb"], z["init_epoch"], z["init_queue"], z["init_log"])
    g2 = GpuBalancer(2 * W + max_e, len(z["init_log"]) + len(z["exp_assign"]) + 64, max_events=max_e + 1)
    g2.load_state(z["init_reg"], z["init_free"], z["init_hb"], z["init_epoch"], z["init_queue"], z["init_log"])
    for t, tk in enumerate(fixture_ticks(z)):
        args = (tk["now"], float(z["tte"]), tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"],
                tk["n_new"])
        a = g.tick(*args, commit=False, compact=True, pinned=True)
        sa = (a["assign"].array(), a["orphans"].copy(), a["evicted"].copy(), a["result"])
        b = g2.tick(*args, commit=False, pinned=False)
        for k, x, y in (("assign", sa[0], b["assign"]), ("orphans", sa[1], b["orphans"]),
                        ("evicted", sa[2], b["evicted"])):
            if not np.array_equal(x, y):
                d = np.nonzero(x[:min(len(x), len(y))] != y[:min(len(x), len(y))])[0]
                print(os.path.basename(path), "tick", t, k, "DIFFER", len(x), len(y), d[:10], x[d[:5]], y[d[:5]])
            else:
                print(os.path.basename(path), "tick", t, k, "ok", len(x))
        g.commit()
        g2.commit()
        if t >= 2:
            break
    g.close()
