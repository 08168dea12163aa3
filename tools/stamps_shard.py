"""Diagnostic: phase stamps of k_emit_shard (exchanged block rows) for rank 0 of a
strong-scaled configs[2] table (or configs[3]: --workload cfg3) at world N, every rank
context on one GPU (libfaasbal_stamps.so, tools/build_all.sh).  Prints per phase the
median shader cycles over the queue blocks and when the blocks start / end (realtime,
from the first block's start):  python tools/stamps_shard.py [--world 8 --reps 30]"""
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
ap.add_argument("--workload", default="tick", choices=("tick", "cfg3"))
args = ap.parse_args()
W, T = (1 << 20, 16_000_000) if args.workload == "cfg3" else (65536, 1_000_000)
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
d = d[:, d[0, :, 13] > 0, :]  # (k_emit_shard_xp: one row per workgroup of 2 queue blocks)
print("world %d, rank 0: %d queue blocks, %d stamped workgroups (stamp rows from %d)" % (args.world, nbq, d.shape[1], SO))
span = (d[:, :, 14].max(axis=1) - d[:, :, 13].min(axis=1)) / 100.0
print("queue-block span (realtime) median %.2f us" % np.median(span))
st0 = (d[:, :, 13] - d[:, :, 13].min(axis=1, keepdims=True)) / 100.0
en0 = (d[:, :, 14] - d[:, :, 13].min(axis=1, keepdims=True)) / 100.0
for qq in (10, 50, 90, 100):
    print("  block start p%d %.2f us, end p%d %.2f us" % (qq, np.median(np.percentile(st0, qq, axis=1)), qq,
                                                      np.median(np.percentile(en0, qq, axis=1))))
prev = 0
for k in (1, 4, 5, 6, 15):  # (the k_plan path stamps 1 after its loads, 5 after the histograms)
    ok = (d[:, :, k] > 0) & (d[:, :, prev] > 0)
    if ok.any():
        dc = (d[:, :, k] - d[:, :, prev])[ok]
        print("  %2d -> %2d  median %6d cyc  p90 %6d" % (prev, k, np.median(dc), np.percentile(dc, 90)))
        prev = k
# k_xscan (large queues): its stamp rows from 3 (nbw + nbf + nbq) + 6000, one per chunk
nch = -(-nbq // 64)
SX = SO + 6000
dx = np.stack([r[: (SX + nch) * 16].reshape(-1, 16).astype(np.int64) for r in rows])[:, SX:SX + nch, :]
if dx.size and (dx[:, :, 13] > 0).all():
    t0 = dx[:, :, 13].min(axis=1, keepdims=True)
    print("k_xscan: %d chunks; start max %.2f us, end max %.2f us (realtime)" % (
        nch, np.median(((dx[:, :, 13] - t0) / 100.0).max(axis=1)), np.median(((dx[:, :, 14] - t0) / 100.0).max(axis=1))))
    prev = 0
    for k in (1, 2, 4, 5, 15):
        dc = (dx[:, :, k] - dx[:, :, prev])
        print("  %2d -> %2d  median %6d cyc  max %6d" % (prev, k, np.median(dc), np.median(dc.max(axis=1))))
        prev = k
# phase 1 (k_scan, rank 0): rows from nbw -- queue blocks, then log tiles, then slot tiles
full = np.stack([r[: (nbw + nbq + nbf + nbw) * 16].reshape(-1, 16).astype(np.int64) for r in rows])
S1 = nbw
roles = {"Q": (S1, S1 + nbq), "F": (S1 + nbq, S1 + nbq + nbf), "W": (S1 + nbq + nbf, S1 + nbq + nbf + nbw)}
e_all = full[:, S1:S1 + nbq + nbf + nbw, 13]
ok = (e_all > 0).all(axis=0)
if ok.any():
    t0 = np.where(e_all > 0, e_all, np.iinfo(np.int64).max).min(axis=1, keepdims=True)
    print("phase-1 k_scan: span %.2f us" % np.median((full[:, S1:S1 + nbq + nbf + nbw, 14].max(axis=1) - t0[:, 0]) / 100.0))
    for name, (lo, hi) in roles.items():
        x = full[:, lo:hi, :]
        live = (x[..., 13] > 0).all(axis=0)
        if hi <= lo or not live.any():
            continue
        x = x[:, live, :]
        ent = (x[..., 13] - t0) / 100.0
        dur = (x[..., 14] - x[..., 13]) / 100.0
        print("  %s %5d blocks: entry p50 +%.2f p90 +%.2f us, duration p50 %.2f p90 %.2f us, 0->1 %d cyc, 1->15 %d cyc"
              % (name, x.shape[1], np.median(ent), np.percentile(ent, 90), np.median(dur), np.percentile(dur, 90),
                 np.median(x[..., 1] - x[..., 0]) if (x[..., 1] > 0).all() else -1,
                 np.median(x[..., 15] - x[..., 1]) if (x[..., 1] > 0).all() else -1))
