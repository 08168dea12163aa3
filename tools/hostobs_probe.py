"""Probe: host-side split of bench.py's host_observed loop at configs[2] (launch, wait,
compact readback into registered pinned arrays; uncommitted relaunches), per call."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
import numpy as np
from faasbal import GpuBalancer, synth

W, T, K = 65536, 1_000_000, 200
st = synth.zipf_state(W=W, seed=0)
g = GpuBalancer(W, 2 * len(st["log"]) + T + 16, max_events=1)
g.load(st)
g.set_compact(True)
g.launch(1000.0, 10.0, n_pending=T)
r = g.wait()
Q = len(st["queue"])
obuf = g.pinned(max(len(st["log"]), 1), np.int64)
ebuf = g.pinned(W, np.int32)
sbuf, cbuf = g.pinned(Q + 16, np.int32), g.pinned(Q + 16, np.uint8)
g.set_compact_out(sbuf, cbuf, obuf, ebuf)
pc = time.perf_counter
acc = np.zeros(4)
for i in range(K + 20):
    t0 = pc()
    g.launch(1000.0, 10.0, n_pending=T)
    t1 = pc()
    g.wait()
    t2 = pc()
    g.outputs_compact(sbuf, cbuf, obuf, ebuf)
    t3 = pc()
    if i >= 20:
        acc += [t1 - t0, t2 - t1, t3 - t2, t3 - t0]
acc /= K
print("configs[2] host_observed us per tick: launch %.1f, wait %.1f, readback %.1f, total %.1f" % tuple(acc * 1e6),
      flush=True)
