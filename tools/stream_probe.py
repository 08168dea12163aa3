"""Probe: host-side time split of the pipelined streaming tick (configs[4] per GPU,
bench.py --workload stream): fb_tick_launch_staged (H2D + enqueue), fb_tick_stage
of the next tick (validation + staging, overlapping the device), fb_tick_wait,
fb_tick_commit -- plus the device time of the tick from the kernel timers."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
import numpy as np
if "--resident" in sys.argv:  # torch before the library (one HIP runtime per process)
    import torch  # noqa: F401
from faasbal import GpuBalancer, synth

W, T, K = 1 << 20, 65536, 30
st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
ticks = synth.stream_ticks(st, n_ticks=K + 6, seed=2, tasks_per_tick=T, results_per_tick=T)
g = GpuBalancer(W, len(st["log"]) + (K + 8) * 2 * T, max_events=max(len(t["ev_kind"]) for t in ticks), device=0)
g.load(st)
if "--eager" in sys.argv:
    g.set_eager_commit(True)
if "--pinned" in sys.argv:  # as bench.py: messages in pinned memory, staging only validates
    for tk in ticks:
        (tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"]) = g.pin_events(
            tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"])
if "--resident" in sys.argv:  # as bench.py's value: every batch in HBM before the loop
    import torch
    for tk in ticks:
        tk["dev"] = [torch.from_numpy(np.ascontiguousarray(tk[k])).to("cuda:0")
                     for k in ("ev_kind", "ev_slot", "ev_val", "ev_ts", "ev_seq")]
carried = 0
acc = np.zeros(5)
pc = time.perf_counter


def stage(tk):
    if "dev" in tk:
        return g.stage_device(tk["now"], *tk["dev"])
    g.stage(tk["now"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"])


stage(ticks[0])
for i, tk in enumerate(ticks[:-1]):
    n = carried + tk["n_new"]
    t0 = pc()
    g.launch_staged(10.0, n)
    t1 = pc()
    stage(ticks[i + 1])
    t2 = pc()
    r = g.wait()
    t3 = pc()
    g.commit()
    t4 = pc()
    carried = n + int(r["n_orphans"]) - int(r["n_assigned"])
    if i >= 5:
        acc += [t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0]
acc /= (len(ticks) - 1 - 5)
print("us per tick: launch_staged %.1f, stage(next) %.1f, wait %.1f, commit %.1f, total %.1f"
      % tuple(acc * 1e6), flush=True)
