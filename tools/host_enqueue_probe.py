"""Probe: is the configs[2] bench loop host-bound?  Times K launches of the idle tick
(bench.py's step) on the host without synchronising, then the wait for the device;
prints host enqueue us per step vs wall us per step."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
from faasbal import GpuBalancer, synth

W, T, K = 65536, 1_000_000, 2000
st = synth.zipf_state(W=W, seed=0)
g = GpuBalancer(W, 2 * len(st["log"]) + T + 16, max_events=1, device=0)
g.load(st)
for _ in range(50):
    g.launch(1000.0, 10.0, n_pending=T)
g.sync()
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(K):
        g.launch(1000.0, 10.0, n_pending=T)
    t1 = time.perf_counter()
    g.sync()
    t2 = time.perf_counter()
    print("host enqueue %.2f us/step, wall %.2f us/step" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6), flush=True)
