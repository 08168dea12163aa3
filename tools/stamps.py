"""Diagnostic: per-phase breakdown of the tick kernels from in-kernel stamps
(libfaasbal_stamps.so, built with -DFAASBAL_STAMPS by tools/build_all.sh).

Slots 0..12 and 15 of a block's row are s_memtime (shader clock, per XCD);
13 / 14 are s_memrealtime (100 MHz, chip-wide) at block entry / exit.
    python tools/stamps.py [--workers 65536 --tasks 1000000 --reps 50]
Run on the GPU box.  Prints, per kernel, the realtime span and, per role, the
block entry offset / duration and the phase deltas in time order."""
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
    ap.add_argument("--stream", action="store_true", help="committed configs[4] ticks with messages")
    ap.add_argument("--hb-frac", type=float, default=0.01)
    ap.add_argument("--dump", default="", help="stream: save the raw stamp rows (npz)")
    ap.add_argument("--fold", action="store_true",
                    help="the tick after a committed tick (its commit folded into k_scan / k_emit2)")
    args = ap.parse_args()
    if args.stream:
        return stream_main(args)
    st = synth.zipf_state(W=args.workers, seed=0)
    W, T = args.workers, args.tasks
    split = args.workers > (1 << 17)  # the library's auto rules (fb_set_path "split_slots" / "logscan")
    fsep = args.workers > (1 << 17)
    g = GpuBalancer(W, 2 * len(st["log"]) + 2 * T + 65536, max_events=1, lib_path=STAMPS_SO)
    g.load(st)
    nbw = -(-W // 256)
    nbf = -(-len(st["log"]) // 2048)
    nbq = max(1, -(-len(st["queue"]) // 256))
    G1 = nbw + nbf + nbq
    acc = []
    for _ in range(args.reps):
        if args.fold:
            g.load(st)
            g.launch(1000.0, 10.0, n_pending=T)
            r0 = g.wait()
            g.commit()  # deferred into the next launch
            # the folded tick's grid: the committed queue and log
            nbf = -(-int(r0["log_head"]) // 2048)
            nbq = max(1, -(-int(r0["queue_len"]) // 256))
            G1 = nbw + nbf + nbq
        g.launch(1000.0, 10.0, n_pending=T)
        g.wait()
        d = g.debug_read()[: 4 * G1 * 16].reshape(4 * G1, 16).astype(np.int64)
        acc.append(d.copy())
    report(np.stack(acc), nbw, nbf, nbq, split, fsep, femit=not split and not fsep)


def stream_main(args):
    """configs[4] ticks (bench.py --workload stream): staged messages, committed
    ticks; the grid of each tick from its queue / log lengths before the launch."""
    W, T = args.workers, 65536
    st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
    n = 5 + args.reps
    ticks = synth.stream_ticks(st, n_ticks=n, seed=2, tasks_per_tick=T, results_per_tick=T, hb_frac=args.hb_frac)
    E = max(len(t["ev_kind"]) for t in ticks)
    g = GpuBalancer(W, len(st["log"]) + (n + 2) * 2 * T, max_events=E, lib_path=STAMPS_SO)
    g.load(st)
    carried = 0
    groups = {}
    for i, tk in enumerate(ticks):
        s = g.read_state(with_log=False)
        Qn, head = len(s["queue"]), int(s["head"])
        Et = len(tk["ev_kind"])
        nbw, nbf, nbq = -(-W // 256), -(-head // 2048), max(1, -(-(Qn + 2 * Et) // 256))
        N = carried + tk["n_new"]
        g.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n_pending=N,
               commit=False)
        r = g.last
        G1 = nbw + nbf + nbq
        if i >= 5:
            d = g.debug_read()[: (3 * G1 + 512 + 131) * 16].reshape(-1, 16).astype(np.int64)
            groups.setdefault((nbw, nbf, nbq), []).append(d.copy())
        g.commit()
        carried = N + int(r["n_orphans"]) - int(r["n_assigned"])
    (nbw, nbf, nbq), acc = max(groups.items(), key=lambda kv: len(kv[1]))
    print("stream ticks with grid nbw %d nbf %d nbq %d: %d of %d" % (nbw, nbf, nbq, len(acc), args.reps))
    if args.dump:
        np.savez_compressed(args.dump, d=np.stack(acc), grid=np.array([nbw, nbf, nbq]))
    report(np.stack(acc), nbw, nbf, nbq, False, True)


def report(d, nbw, nbf, nbq, split, fsep, femit=False):
    """d: reps x rows x 16 stamps.  femit: fused one-GPU ticks (k_scan without log
    blocks; k_emit2's log role one workgroup per tile, then the slot tiles four per
    workgroup)."""
    G1 = nbw + nbf + nbq
    S = nbw  # k_scan rows start here
    E0 = G1 if split else G1 + nbw  # k_emit rows start here
    if fsep:
        # k_scan = W + Q roles, k_logscan (<= 256 rows from 3*G1), k_plan (rows from 3*G1 + 512), k_emit
        E0 = 2 * nbw + nbf + nbq
        ls = min(256, -(-nbf // 16))
        L0, P0 = 3 * G1, 3 * G1 + 512
        nplan = 3 + 128
        kernels = {"scan": (S, S + nbw + nbq), "logscan": (L0, L0 + ls), "plan": (P0, P0 + nplan),
                   "emit": (E0, E0 + G1)}
        roles = {"scan.Q": (S, S + nbq), "scan.W": (S + nbq, S + nbq + nbw), "logscan": (L0, L0 + ls),
                 "plan": (P0, P0 + nplan)}
    elif split:
        kernels = {"slots": (0, nbw), "scan": (S, S + nbf + nbq), "emit": (E0, E0 + G1)}
        roles = {"slots": (0, nbw), "scan.Q": (S, S + nbq), "scan.F": (S + nbq, S + nbq + nbf)}
    else:
        kernels = {"scan": (S, S + nbf + nbw + nbq), "emit": (E0, E0 + G1)}
        roles = {"scan.Q": (S, S + nbq), "scan.F": (S + nbq, S + nbq + nbf), "scan.W": (S + nbq + nbf, S + G1)}
    nbf4, nbw4 = -(-nbf // 4), -(-nbw // 4)  # k_emit2: one wave per compaction tile
    if femit:
        kernels["scan"] = (S, S + nbq + nbw)
        roles = {"scan.Q": (S, S + nbq), "scan.W": (S + nbq, S + nbq + nbw)}
        nbf4 = nbf  # one log workgroup per tile
    roles.update({"emit.Q": (E0, E0 + nbq), "emit.F": (E0 + nbq, E0 + nbq + nbf4),
                  "emit.W": (E0 + nbq + nbf4, E0 + nbq + nbf4 + nbw4)})
    starts = {}
    for kern, (lo, hi) in list(kernels.items()):
        live = (d[:, lo:hi, 13] > 0).all(axis=0)
        if not live.any():
            del kernels[kern]
            continue
        hi = lo + int(np.nonzero(live)[0].max()) + 1
        kernels[kern] = (lo, hi)
        ent, ext = d[:, lo:hi, 13], d[:, lo:hi, 14]
        starts[kern] = ent.min(axis=1)
        span = (ext.max(axis=1) - ent.min(axis=1)) / 100.0
        spread = (ent.max(axis=1) - ent.min(axis=1)) / 100.0
        print("%-6s span %.2f us (median), entry spread %.2f us" % (kern, np.median(span), np.median(spread)))
        # resident blocks: mean (block-time / span) and the peak, first rep
        e0, x0 = ent[0], ext[0]
        ev = np.concatenate([np.stack([e0, np.ones_like(e0)], 1), np.stack([x0, -np.ones_like(x0)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        print("       resident blocks: mean %.0f, peak %d" % ((x0 - e0).sum() / max(1, x0.max() - e0.min()),
                                                              int(np.cumsum(ev[:, 1]).max())))
        # blocks entering / leaving per microsecond (first rep)
        nb = int((x0.max() - e0.min()) // 100) + 1
        hin = np.bincount(((e0 - e0.min()) // 100).astype(int), minlength=nb)
        hout = np.bincount(((x0 - e0.min()) // 100).astype(int), minlength=nb)
        print("       entering per us:", " ".join(str(int(v)) for v in hin))
        print("       leaving  per us:", " ".join(str(int(v)) for v in hout))
        top = d[:, lo:hi, 12]
        if (top > 0).all():
            # realtime at the top of the kernel, before the argument copy
            tsp = (top.max(axis=1) - top.min(axis=1)) / 100.0
            lag = np.median((ent - top) / 100.0, axis=1)
            print("       top-of-kernel spread %.2f us, top -> entry stamp median %.2f us" % (np.median(tsp),
                                                                                          np.median(lag)))
    ks = list(kernels)
    for a, b in zip(ks[:-1], ks[1:]):
        gap = (starts[b] - d[:, kernels[a][0]:kernels[a][1], 14].max(axis=1)) / 100.0
        print("gap %s end -> %s first entry: %.2f us" % (a, b, np.median(gap)))
    for name, (lo, hi) in roles.items():
        live = (d[:, lo:hi, 13] > 0).all(axis=0)
        if not live.any():
            continue
        hi = lo + int(np.nonzero(live)[0].max()) + 1
        x = d[:, lo:hi, :]
        kern = name.split(".")[0]
        off = (x[..., 13] - starts[kern][:, None]) / 100.0
        dur = (x[..., 14] - x[..., 13]) / 100.0
        print("%-7s %4d blocks: entry +%.2f us (p90 %.2f), duration %.2f us (p90 %.2f)" % (
            name, hi - lo, np.median(off), np.percentile(off, 90), np.median(dur), np.percentile(dur, 90)))
        used = [k for k in range(12) if (x[..., k] > 0).all()] + [15]
        med = {k: np.median(x[..., k] - x[..., 0]) for k in used}
        order = sorted(used, key=lambda k: med[k])
        for a, b in zip(order[:-1], order[1:]):
            dt = (x[..., b] - x[..., a]).ravel()
            print("      %2d->%2d  median %7d cyc  p90 %7d" % (a, b, np.median(dt), np.percentile(dt, 90)))


if __name__ == "__main__" and "--hist" not in sys.argv and "--xcd" not in sys.argv:
    main()


def entry_histogram(workers=65536, tasks=1_000_000, reps=20):
    """Diagnostic: sorted top-of-kernel offsets of k_scan's blocks (first rep) in 10 bins."""
    st = synth.zipf_state(W=workers, seed=0)
    g = GpuBalancer(workers, 2 * len(st["log"]) + tasks + 16, max_events=1, lib_path=STAMPS_SO)
    g.load(st)
    nbw, nbf, nbq = -(-workers // 256), -(-len(st["log"]) // 2048), max(1, -(-len(st["queue"]) // 256))
    for _ in range(reps):
        g.launch(1000.0, 10.0, n_pending=tasks)
        g.wait()
    d = g.debug_read()[: 4 * (nbw + nbf + nbq) * 16].reshape(-1, 16).astype(np.int64)
    top = d[nbw:nbw + nbq + nbf + nbw, 12]
    rel = (top - top.min()) / 100.0
    roles = np.array(["Q"] * nbq + ["F"] * nbf + ["W"] * nbw)
    order = np.argsort(rel)
    print("k_scan top-of-kernel offsets (us) by block-id decile:")
    for dec in range(10):
        lo, hi = dec * len(rel) // 10, (dec + 1) * len(rel) // 10
        print("  blocks %4d-%4d: median +%.2f  max +%.2f" % (lo, hi - 1, np.median(rel[lo:hi]), rel[lo:hi].max()))
    print("  latest 20 blocks:", [(int(i), roles[i], round(float(rel[i]), 2)) for i in order[-20:]])


if __name__ == "__main__" and "--hist" in sys.argv:
    entry_histogram()


def xcd_table(workers=65536, tasks=1_000_000, reps=30):
    """Diagnostic: per XCD (block id mod 8) the median top-of-kernel offset and the
    median exit offset of k_scan and k_emit2 blocks, relative to the kernel's first top stamp."""
    st = synth.zipf_state(W=workers, seed=0)
    g = GpuBalancer(workers, 2 * len(st["log"]) + tasks + 16, max_events=1, lib_path=STAMPS_SO)
    g.load(st)
    nbw, nbf, nbq = -(-workers // 256), -(-len(st["log"]) // 2048), max(1, -(-len(st["queue"]) // 256))
    G1 = nbw + nbf + nbq
    acc = []
    for _ in range(reps):
        g.launch(1000.0, 10.0, n_pending=tasks)
        g.wait()
        acc.append(g.debug_read()[: 4 * G1 * 16].reshape(-1, 16).astype(np.int64).copy())
    d = np.stack(acc)
    E0 = G1 + nbw
    ne = nbq + -(-nbf // 4) + -(-nbw // 4)
    for name, lo, n in (("scan", nbw, G1), ("emit", E0, ne)):
        x = d[:, lo:lo + n]
        t0 = x[..., 12].min(axis=1)[:, None]
        top = (x[..., 12] - t0) / 100.0
        ext = (x[..., 14] - t0) / 100.0
        xcd = np.arange(n) % 8
        print("%s: per block-id mod 8: median top offset / median exit offset (us)" % name)
        print("   " + "  ".join("%d: %.2f/%.2f" % (k, np.median(top[:, xcd == k]), np.median(ext[:, xcd == k]))
                               for k in range(8)))
        if name == "scan":
            prev_end = None
        # gap from the previous kernel's last exit
    print("emit end -> next scan top: measured per rep is not available (one tick per rep)")


if __name__ == "__main__" and "--xcd" in sys.argv:
    xcd_table()
