"""Probe: per-rank device time of the sharded tick at world N,
all N rank contexts on ONE GPU (exchange summed on-device, no RCCL): what one
rank of the N-GPU bench computes per tick, minus the all-reduce.  strong (default,
bench.py --gpus N): the configs[2] table of 64K workers / 1M tasks split N ways;
weak: N x 64K workers / N x 1M tasks.  Reports rank 0 and the slowest rank.

    python tools/shard_probe.py [--world 2 4 8 --reps 50 --scaling strong --workload tick|cfg3]
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
    ap.add_argument("--scaling", default="strong", choices=("strong", "weak"))
    ap.add_argument("--workload", default="tick", choices=("tick", "cfg3"),
                    help="tick: configs[2] (64K workers, 1M tasks); cfg3: configs[3] (1M workers, 16M tasks)")
    ap.add_argument("--gated", action="store_true",
                    help="per rank: phase 1, exchange copy and phase 2 back to back behind the timing gate")
    args = ap.parse_args()
    for world in args.world:
        k = world if args.scaling == "weak" else 1
        W0, T0 = (1 << 20, 16_000_000) if args.workload == "cfg3" else (65536, 1_000_000)
        W, T = W0 * k, T0 * k
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
            return tot

        for _ in range(5):
            tick()
        # the summed exchange of two consecutive ticks: the records alternate between two
        # copies by exchange parity, so the contents repeat with period 2
        tots = [tick(), tick()]  # phase 2's input (the summed exchange) of two consecutive ticks
        rep = [0]

        def tick_gated():
            # each rank alone, its phases back to back on the device behind the timing gate:
            # phase 1, the exchange's summed contents (this idle tick's, identical every other
            # repetition) copied in on the rank's stream, phase 2 -- no host pacing between
            tot = tots[rep[0] % 2]
            rep[0] += 1
            for b in bals:
                b.timing_gate(True)
                b.launch(1000.0, 10.0, n_pending=T)
                with torch.cuda.stream(b.stream):
                    b.exchange().copy_(tot)
                b.cont()
                b.timing_gate(False)
                b.wait()

        for b in bals:
            b.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            (tick_gated if args.gated else tick)()
        dt = (time.perf_counter() - t0) / args.reps
        pers = []
        for b in bals:
            kt = b.timing_read()
            pers.append({k: round(ms / args.reps * 1e3, 2) for k, (ms, n) in kt.items()})
        slow = max(range(world), key=lambda r: sum(pers[r].values()))
        print("%s%s %s world %d: rank-0 device us per tick %s (sum %.1f); slowest rank %d: sum %.1f; exchange %d B, "
              "serial wall %.0f us" % (args.workload, " gated" if args.gated else "", args.scaling, world, pers[0], sum(pers[0].values()), slow,
                                       sum(pers[slow].values()), bals[0].exchange().numel(), dt * 1e6), flush=True)
        for b in bals:
            b.timing_enable(False)
            b.close()


if __name__ == "__main__":
    main()
