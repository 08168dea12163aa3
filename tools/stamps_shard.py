"""Diagnostic: phase stamps of k_emit_shard (exchanged block rows) for rank 0 of a
strong-scaled configs[2] table at world N, every rank context on one GPU
(libfaasbal_stamps.so, tools/build_all.sh).  Prints per phase the median shader
cycles over the queue blocks:  python tools/stamps_shard.py [--world 8 --reps 30]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
import torch  # noqa: E402,F401

from faasbal import synth  # noqa: E402
from faasbal.sharded import ShardedBalancer, split_state  # noqa: E402

STAMPS_SO = os.path.join(REPO, "distributed-faas_amd", "faasbal", "libfaasbal_stamps.so")

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--reps", type=int, default=30)
args = ap.parse_args()
W, T = 65536, 1_000_000
st = synth.zipf_state(W=W, seed=0)
F = len(st["log"])
bals = [ShardedBalancer(r, args.world, W, 2 * F // args.world + T + 16, max_events=1, lib_path=STAMPS_SO)
        for r in range(args.world)]
for b in bals:
    b.load(st)
rows = []
for it in range(args.reps + 3):
    for b in bals:
        b.launch(1000.0, 10.0, n_pending=T)
        b.sync()
    tot = bals[0].exchange().clone()
    for b in bals[1:]:
        tot += b.exchange()
    for b in bals:
        b.exchange().copy_(tot)
    torch.cuda.synchronize()
    for b in bals:
        b.cont()
        b.wait()
    if it >= 3:
        rows.append(bals[0].debug_read().copy())
p0 = split_state(st, args.world, 0)  # (every rep is the same uncommitted tick)
nbq = max(1, -(-(len(st["queue"])) // 256))
nbw = max(1, -(-int(p0["n"]) // 256))
nbf = -(-len(p0["log_slot"]) // 2048)
SO = 3 * (nbw + nbf + nbq)
d = np.stack([r[: (SO + nbq) * 16].reshape(-1, 16).astype(np.int64) for r in rows])[:, SO:SO + nbq, :]
print("world %d, rank 0: %d queue blocks (stamp rows from %d)" % (args.world, nbq, SO))
span = (d[:, :, 14].max(axis=1) - d[:, :, 13].min(axis=1)) / 100.0
print("queue-block span (realtime) median %.2f us" % np.median(span))
prev = 0
for k in (1, 4, 5, 6, 15):
    ok = (d[:, :, k] > 0) & (d[:, :, prev] > 0)
    if ok.any():
        dc = (d[:, :, k] - d[:, :, prev])[ok]
        print("  %2d -> %2d  median %6d cyc  p90 %6d" % (prev, k, np.median(dc), np.percentile(dc, 90)))
        prev = k
