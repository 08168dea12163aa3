"""Probe: host cost of one configs[2] tick launch vs its device time.

    python tools/launch_probe.py [--steps 400]

Times K back-to-back GpuBalancer.launch() calls (host side only, then the
drain), the same through a bare ctypes call with prebuilt arguments, and the
device time per tick -- to tell whether bench.py's wall per step is bound by
the host (Python + HIP launch) or by the kernels.
"""
import argparse
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))

from faasbal import GpuBalancer, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    W, T = 65536, 1_000_000
    st = synth.zipf_state(W=W, seed=0)
    F = len(st["log"])
    g = GpuBalancer(W, 2 * F + T + 16, max_events=1, device=0)
    g.load(st)
    for _ in range(20):
        g.launch(1000.0, 10.0, n_pending=T)
    g.sync()
    K = a.steps
    for rep in range(2):
        t0 = time.perf_counter()
        for _ in range(K):
            g.launch(1000.0, 10.0, n_pending=T)
        t1 = time.perf_counter()
        g.sync()
        t2 = time.perf_counter()
        print("python launch: host %.2f us/call, wall %.2f us/tick" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6))
        f = g.lib.fb_tick_launch
        h = g.h
        args = (h, C.c_double(1000.0), C.c_double(10.0), 0, None, None, None, None, None, T)
        t0 = time.perf_counter()
        for _ in range(K):
            f(*args)
        t1 = time.perf_counter()
        g.sync()
        t2 = time.perf_counter()
        print("bare ctypes:   host %.2f us/call, wall %.2f us/tick" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6))
    g.timing_enable(True)
    for _ in range(K):
        g.launch(1000.0, 10.0, n_pending=T)
    kt = g.timing_read()
    g.timing_enable(False)
    print("device us per tick:", {k: round(ms / n * 1e3, 2) for k, (ms, n) in kt.items()})


if __name__ == "__main__":
    main()
