"""Diagnostic: per-phase cycle breakdown of the tick kernels from in-kernel
s_memtime stamps (libfaasbal_stamps.so, built with -DFAASBAL_STAMPS).

    python tools/stamps.py [--workers 65536 --tasks 1000000 --reps 50]
Run on the GPU box; prints median/max cycles per phase and role."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
from faasbal import synth  # noqa: E402
from faasbal.balancer import GpuBalancer  # noqa: E402

STAMPS_SO = os.path.join(REPO, "distributed-faas_amd", "faasbal", "libfaasbal_stamps.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=65536)
    ap.add_argument("--tasks", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    st = synth.zipf_state(W=args.workers, seed=0)
    W, T = args.workers, args.tasks
    g = GpuBalancer(W, 2 * len(st["log"]) + T + 16, max_events=1, lib_path=STAMPS_SO)
    g.load(st)
    nbw = -(-W // 256)
    nbf = -(-len(st["log"]) // 2048)
    nbq = max(1, -(-len(st["queue"]) // 256))
    G1 = nbw + nbf + nbq
    acc = []
    for _ in range(args.reps):
        g.launch(1000.0, 10.0, n_pending=T)
        g.wait()
        d = g.debug_read()[: 2 * G1 * 16].reshape(2 * G1, 16).astype(np.int64)
        acc.append(d.copy())
    d = np.stack(acc)  # reps x blocks x 16
    roles = {"slots": (0, nbw), "scan.F": (nbw, nbw + nbf), "scan.Q": (nbw + nbf, G1),
             "emit.Q": (G1, G1 + nbq), "emit.F": (G1 + nbq, G1 + nbq + nbf), "emit.W": (G1 + nbq + nbf, 2 * G1)}
    for kern, (lo, hi) in (("slots", (0, nbw)), ("scan", (nbw, G1)), ("emit", (G1, 2 * G1))):
        span = d[:, lo:hi, 15].max(axis=1) - d[:, lo:hi, 0].min(axis=1)
        start_spread = d[:, lo:hi, 0].max(axis=1) - d[:, lo:hi, 0].min(axis=1)
        print("%s: kernel span median %d cycles, block start spread %d" % (kern, np.median(span), np.median(start_spread)))
    for name, (lo, hi) in roles.items():
        x = d[:, lo:hi, :]
        used = [k for k in range(13) if (x[..., k] > 0).all()] + [15]
        if (x[..., 13] > 0).all() and (x[..., 14] > 0).all():
            rt = (x[..., 14] - x[..., 13]).ravel() / 100.0  # s_memrealtime: 100 MHz
            cy = (x[..., 15] - x[..., 0]).ravel()
            print("   realtime entry->exit median %.2f us; shader clock %.2f GHz" % (np.median(rt), np.median(cy / rt) / 1e3))
        print(name, "blocks", hi - lo, "stamps", used)
        for a, b in zip(used[:-1], used[1:]):
            dt = (x[..., b] - x[..., a]).ravel()
            print("   %2d->%2d  median %7d  p90 %7d  max %7d" % (a, b, np.median(dt), np.percentile(dt, 90), dt.max()))
        # completion time relative to the kernel's first block start
        kl, kh = (0, nbw) if name == "slots" else ((nbw, G1) if name.startswith("scan") else (G1, 2 * G1))
        first = d[:, kl:kh, 0].min(axis=1)[:, None]
        end = (x[..., 15] - first).ravel()
        print("   end-from-kernel-start median %d max %d" % (np.median(end), end.max()))


if __name__ == "__main__":
    main()
