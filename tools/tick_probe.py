"""Probe: host issue time vs device time of the configs[2] tick (diagnostic)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
import ctypes as C
from faasbal import GpuBalancer, synth

st = synth.zipf_state(W=65536, seed=0)
F = len(st["log"]); T = 1_000_000
g = GpuBalancer(65536, 2 * F + T + 16, max_events=1, device=0)
g.load(st)
for _ in range(20):
    g.launch(1000.0, 10.0, n_pending=T)
g.sync()
K = 400
t0 = time.perf_counter()
for _ in range(K):
    g.launch(1000.0, 10.0, n_pending=T)
t1 = time.perf_counter()
g.sync()
t2 = time.perf_counter()
print("python launch: issue %.2f us/tick, wall %.2f us/tick" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6))
fn = g.lib.fb_tick_launch
h = g.h
t0 = time.perf_counter()
for _ in range(K):
    fn(h, 1000.0, 10.0, 0, None, None, None, None, None, T)
t1 = time.perf_counter()
g.sync()
t2 = time.perf_counter()
print("raw ctypes launch: issue %.2f us/tick, wall %.2f us/tick" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6))
