"""Model of k_emit2's task-store bytes at configs[2] (VERDICT r3 ask 4).

Refuted by measurement (profiles/NOTES_r04.md): granule-aligned block runs wrote the same
PMC bytes at configs[3], so run ends merge in L2; kept as the record of the hypothesis.

Every wave stores its active lanes' tasks of a round as one contiguous run of 4-byte
slots (task index base(r) + its rank among the wave's active lanes); a run starts and
ends inside a memory granule that the neighbouring wave's run shares.  If each store
request leaves L2 as whole granules, the bytes written are the runs rounded out to
granules.  Prints, per granule size, the bytes of the per-wave runs and of per-block
runs (the same tasks staged through LDS and stored by the block as one run per round)
against the 4 B per task of the tick.

    python tools/emit_write_model.py [--workers 65536] [--tasks 1000000]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-faas_amd"))
from faasbal import synth  # noqa: E402


def runs_bytes(c, S, L, width, g):
    """Bytes of the round runs of groups of `width` positions, rounded out to g-byte granules."""
    n = (len(c) + width - 1) // width * width
    cp = np.zeros(n, np.int64)
    cp[:len(c)] = c
    grp = cp.reshape(-1, width)
    tot = runs = 0
    for r in range(L + 1):
        k = (grp > r).sum(1)
        before = np.concatenate([[0], np.cumsum(k)[:-1]])
        start = (S[r] + before) * 4
        end = start + 4 * k
        m = k > 0
        tot += int(np.sum((end[m] + g - 1) // g - start[m] // g)) * g
        runs += int(m.sum())
    return tot, runs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=65536)
    ap.add_argument("--tasks", type=int, default=1_000_000)
    args = ap.parse_args()
    st = synth.zipf_state(W=args.workers, seed=0)
    q = np.asarray(st["queue"])
    alive_slot = st["reg"].astype(bool) & ~((1000.0 - st["hb"]) > 10.0)
    c = np.where(alive_slot[q], np.maximum(st["free"][q], 1), 0).astype(np.int64)
    dead = st["reg"].astype(bool) & ((1000.0 - st["hb"]) > 10.0)
    log = np.asarray(st["log"])
    O = int(np.sum((log >= 0) & dead[np.clip(log, 0, None)]))
    N = O + args.tasks
    A = np.array([(c > r).sum() for r in range(int(c.max()) + 1)])
    S = np.concatenate([[0], np.cumsum(A)])
    L = int(np.searchsorted(S, N, side="right") - 1)
    ideal = 4 * int(S[L])
    print("Q %d, O %d, N %d, fill level L %d, tasks in full rounds %d (%.3f MB of slots)"
          % (len(q), O, N, L, S[L], ideal / 1e6))
    for g in (32, 64, 128):
        for width, what in ((64, "per wave"), (256, "per block")):
            b, runs = runs_bytes(c, S, L, width, g)
            print("  %3d-B granules, %-9s runs: %6d runs, %.3f MB (+%.3f MB)" % (g, what, runs, b / 1e6, (b - ideal) / 1e6))


if __name__ == "__main__":
    main()
