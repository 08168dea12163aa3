"""Probe: per-rank device time of the sharded tick at world N,
all N rank contexts on ONE GPU (exchange summed on-device, no RCCL): what one
rank of the N-GPU weak-scaling bench computes per tick, minus the all-reduce.

    python tools/shard_probe.py [--world 2 4 8 --reps 50]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))

import torch  # noqa: E402

from faasbal import synth  # noqa: E402
from faasbal.sharded import ShardedBalancer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    for world in args.world:
        W, T = 65536 * world, 1_000_000 * world
        st = synth.zipf_state(W=W, seed=0)
        F = len(st["log"])
        bals = [ShardedBalancer(r, world, W, 2 * F // world + T + 16, max_events=1) for r in range(world)]
        for b in bals:
            b.load(st)

        def tick():
            # ranks one after another, each alone on the GPU (as on its own GPU)
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

        for _ in range(5):
            tick()
        for b in bals:
            b.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            tick()
        dt = (time.perf_counter() - t0) / args.reps
        kt = bals[0].timing_read()
        per = {k: round(ms / args.reps * 1e3, 2) for k, (ms, n) in kt.items()}
        print("world %d: rank-0 device us per tick %s (sum %.1f), exchange %d B, serial wall %.0f us"
              % (world, per, sum(per.values()), bals[0].exchange().numel(), dt * 1e6), flush=True)
        for b in bals:
            b.timing_enable(False)
            b.close()


if __name__ == "__main__":
    main()
