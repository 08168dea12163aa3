"""Probe: host enqueue rate of the sharded tick vs its device time (one rank
context of world N on one GPU, no collective: the exchange is left as phase 1
wrote it, so results are not meaningful -- only the timing is).

    python tools/host_rate_probe.py [--world 1 2 8 --reps 300]

Prints, per world: wall us per tick with K ticks queued back to back (host
enqueue + device), the host-only cost of the enqueue calls, and the device sum.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))

import torch  # noqa: E402

from faasbal import GpuBalancer, synth  # noqa: E402
from faasbal.sharded import ShardedBalancer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[1, 2, 8])
    ap.add_argument("--reps", type=int, default=300)
    args = ap.parse_args()
    for world in args.world:
        W, T = 65536 * world, 1_000_000 * world
        st = synth.zipf_state(W=W, seed=0)
        F = len(st["log"])
        if world == 1:
            b = GpuBalancer(W, 2 * F + T + 16, max_events=1)
            b.load(st)

            def step():
                b.launch(1000.0, 10.0, n_pending=T)
        else:
            b = ShardedBalancer(0, world, W, 2 * F // world + T + 16, max_events=1)
            b.load(st)
            acc = [0.0, 0.0, 0.0]
            pc = time.perf_counter

            def step():
                # stand-in for the collective's host call: one tiny torch op on the stream
                t0 = pc()
                b.launch(1000.0, 10.0, n_pending=T)
                t1 = pc()
                with torch.cuda.stream(b.stream):
                    b.exchange()[:1].add_(0)
                t2 = pc()
                b.cont()
                t3 = pc()
                acc[0] += t1 - t0
                acc[1] += t2 - t1
                acc[2] += t3 - t2
        for _ in range(20):
            step()
        b.sync()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            step()
        th = time.perf_counter() - t0
        b.sync()
        dt = time.perf_counter() - t0
        b.timing_enable(True)
        for _ in range(args.reps):
            step()
        kt = b.timing_read()
        b.timing_enable(False)
        b.sync()
        per = {k: round(ms / args.reps * 1e3, 2) for k, (ms, n) in kt.items()}
        if world > 1:
            n = 2 * args.reps + 20
            print("  host split us/tick: launch %.1f, torch op on stream %.1f, cont %.1f"
                  % tuple(x / n * 1e6 for x in acc), flush=True)
        print("world %d: wall %.1f us/tick, host enqueue %.1f us/tick, device %s sum %.1f"
              % (world, dt / args.reps * 1e6, th / args.reps * 1e6, per, sum(per.values())), flush=True)


if __name__ == "__main__":
    main()
