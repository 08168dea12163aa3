"""Benchmark: task assignment decisions/s of the HIP push balancer.

Workload (BASELINE.json configs[2], the headline): one tick over
1M pending tasks x 64K workers, Zipf(1.5) loads capped at 32, 5 % of workers
past the heartbeat timeout (evicted, their in-flight tasks redistributed
first).  A step = one full tick (events -> purge -> orphans -> water-filling
dispatch -> next state) over that synthetic state, resident in HBM; the tick
is functional (reads the committed state, writes outputs and the next state
to separate buffers), so K steps recompute the same tick without cached work.

Prints one JSON line (rank 0).  Multi-GPU: see DESIGN.md §6.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


def tick_bytes(W, Q, F, O, N, E=0):
    """SURVEY.md §8(d) algorithmic bytes of one tick."""
    return 16 * W + 8 * W + 4 * (N - O) + 4 * F + 8 * O + 17 * E


def emit_bytes(W, Q, F, O, N, Qn_out, n_evicted, log_in_emit=False):
    """Algorithmic bytes of one k_emit launch.  Queue role, per LRU
    position: its c, heartbeat and slot (4+8+4 B read), next free count and
    queued flag of its worker (4+1 B written); per task its slot (4 B); per
    next-queue entry slot, free count and heartbeat (4+4+8 B).  Log role: the
    orphan flags (1 bit per in-flight entry) and the orphan ids (8 B each) --
    or, when the emit flags the orphans itself (fused one-GPU ticks), every
    in-flight entry's slot (4 B) and the died bitmap (W/8 B) once.  Slot role:
    the slot status byte and the evicted ids (4 B each)."""
    log = 4 * F + W // 8 if log_in_emit else F // 8
    return 4 * N + 21 * Q + 16 * Qn_out + log + 8 * O + W + 4 * n_evicted


def scan_bytes(W, Q, F, logscan=False):
    """Algorithmic bytes of one k_scan launch: slot role per slot its record
    (registered 1 + {hb, epoch} 16 + free 4 B) in, status byte, next free count
    and queued flag (1+4+1 B) out; queue role per LRU position its ride-along
    free count and heartbeat (4+8 B) in, c and heartbeat (4+8 B) out; log role
    (unless k_logscan runs it) per in-flight entry its slot (4 B), its worker's
    16-byte record and 1 bit of orphan flags."""
    b = 27 * W + 24 * Q
    if not logscan:
        b += 20 * F + F // 8
    return b


def logscan_bytes(W, F):
    """k_logscan: per in-flight entry its slot (4 B) and 1 bit of orphan flags; the
    died bitmap (W/8 B) once."""
    return 4 * F + F // 8 + W // 8


def emit_deque_bytes(Q, N, Qn_out):
    """k_emit in deque mode (start()): task writes (4 B/task), per deque entry its
    c and slot (4+4) and token record {j, m, q, k} (16), its worker's count
    update (4+4) and K_L (4); next deque entry + rank (4+4) and the per-slot
    token count (4+4)."""
    return 4 * N + 36 * Q + 16 * Qn_out


def emit_shard_bytes(Q, own_q, F_local, O_local, n_local, Qn_out):
    """Algorithmic bytes of k_emit_shard on one rank: c8 exchange byte + queue
    slot read + next-queue write per LRU position (1+4+4), own tasks (slot and
    global sequence, 8 B), own c_arr read + free_processes write (8 B per own
    queued worker), log shard re-read for orphan compaction and orphan ids."""
    return 9 * Q + 4 * Qn_out + 8 * n_local + 8 * own_q + 4 * F_local + 8 * O_local


def cpu_baseline(st, T, budget_s=10.0):
    """The oracle (C restatement of the reference loop, 1 core) on a bounded
    prefix of the same tick: the loop as written (O(W) purge per iteration)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from oracle import Oracle
    W = len(st["reg"])
    cap = len(st["log"]) * 2 + T + 16
    # calibrate the prefix length on a short run, then time ~budget_s
    o = Oracle(W, cap, purge_mode=0)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    t0 = time.perf_counter()
    o.tick(1000.0, 10.0, [], [], [], [], [], T, dispatch_limit=200)
    dt = time.perf_counter() - t0
    n = int(max(200, min(T, 200 * budget_s / max(dt, 1e-6))))
    o = Oracle(W, cap, purge_mode=0)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    t0 = time.perf_counter()
    out = o.tick(1000.0, 10.0, [], [], [], [], [], T, dispatch_limit=n)
    dt = time.perf_counter() - t0
    rate = len(out["assign"]) / dt
    # purge-once variant (same results, no redundant O(W) purges): full tick
    o = Oracle(W, cap, purge_mode=1)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    t0 = time.perf_counter()
    full = o.tick(1000.0, 10.0, [], [], [], [], [], T)
    dt1 = time.perf_counter() - t0
    return dict(value=rate, unit="assignments/s", cores=1, kind="port",
                sample="first %d dispatches of the configs[2] tick, loop as written (O(W) purge per "
                       "iteration), oracle/push_oracle.c; host nproc=%d" % (len(out["assign"]), os.cpu_count()),
                purge_once_value=len(full["assign"]) / dt1,
                purge_once_sample="whole tick (%d dispatches), purge skipped when provably idempotent"
                                  % len(full["assign"]))


def cpu_baseline_deque(st, T, budget_s=10.0):
    """oracle/deque_oracle.c (the start() loop as written, 1 core) on the whole tick."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from oracle import DequeOracle
    W = len(st["reg"])
    o = DequeOracle(W, len(st["log"]) + T + 16)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    t0 = time.perf_counter()
    out = o.tick(1000.0, 0.0, [], [], [], [], [], T)
    dt = time.perf_counter() - t0
    return dict(value=len(out["assign"]) / dt, unit="assignments/s", cores=1, kind="port",
                sample="whole tick (%d dispatches), start() loop as written, oracle/deque_oracle.c; host nproc=%d"
                       % (len(out["assign"]), os.cpu_count()))


def bench_stream(args, dist=None, world=1, rank=0, dev=0):
    """BASELINE.json configs[4]: 1M workers, every tick 64K new tasks, 64K results
    of in-flight tasks, 1K re-registrations, 10K heartbeats; the clock advances
    10 ms per tick so silent workers expire (churn) and their in-flight tasks are
    redistributed.  Ticks are committed (state evolves); the timed region holds K
    whole ticks.  One GPU: host staging of the events (tick i+1's overlapping
    tick i on the device), the launch, the wait for the results and the commit.
    N GPUs (configs[4] as stated, "8 MI355X"): the 1M-worker table sharded by
    worker-id range, every rank receives the tick's whole message batch, phase 1
    -> the exchange all-reduce (RCCL) -> phase 2 -> wait -> commit on every rank."""
    from faasbal import GpuBalancer, synth
    W = args.workers if args.workers != 65536 else 1 << 20
    T = 65536
    K, Wu = min(args.steps, 50), min(args.warmup, 5)  # 64K distinct results per tick from the initial log
    st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
    ticks = synth.stream_ticks(st, n_ticks=Wu + 2 * K, seed=2, tasks_per_tick=T, results_per_tick=T,
                               hb_frac=args.hb_frac, dt=0.0 if args.stream_quiet else 0.01)
    if args.stream_quiet:
        # no churn: no re-registrations and a clock that ages nobody, so no registration dies
        # (the log scan is skipped on window ticks)
        for tk in ticks:
            keep = tk["ev_kind"] != synth.EV_REGISTER
            for k in ("ev_kind", "ev_slot", "ev_val", "ev_ts", "ev_seq"):
                tk[k] = tk[k][keep]
    E = max(len(t["ev_kind"]) for t in ticks)
    cap = len(st["log"]) + (Wu + 2 * K + 2) * 2 * T
    carried = [0]
    stats = dict(assigned=0, orphans=0, evicted=0, events=0)
    pcie = None
    if world == 1:
        import torch
        g = GpuBalancer(W, cap, max_events=E, device=0)
        mode = "pageable" if args.pageable_events else args.events

        def prep(mode):
            # hbm: every tick's batch copied into HBM before the timed region (the contract's
            # value: inputs resident); pinned: the producer writes each tick's messages into
            # pinned host memory (as the dispatcher's parse loop can) and the tick's H2D
            # copies are inside the timed region; pageable: numpy arrays, staged by copy
            for tk in ticks:
                arrs = [tk[k] for k in ("ev_kind", "ev_slot", "ev_val", "ev_ts", "ev_seq")]
                if mode == "hbm":
                    tk["dev"] = [torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0") for a in arrs]
                elif mode == "pinned":
                    tk["pin"] = g.pin_events(*arrs)

        def stage(tk):
            if mode == "hbm":
                g.stage_device(tk["now"], *tk["dev"])
            elif mode == "pinned":
                g.stage(tk["now"], *tk["pin"])
            else:
                g.stage(tk["now"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"])

        def loop(i0, i1):
            # ticks [i0, i1), tick i0's messages staged: launch tick i on its staged messages,
            # stage tick i+1's while the device runs tick i (double-buffered), wait, commit,
            # launch tick i+1 at once -- the bookkeeping of tick i comes after (off the path
            # between one tick's end and the next one's first kernel)
            out = []
            n = carried[0] + ticks[i0]["n_new"]
            g.launch_staged(10.0, n)
            if i0 + 1 < len(ticks):
                stage(ticks[i0 + 1])
            for i in range(i0, i1):
                r = g.wait()
                g.commit()
                carried[0] = n + int(r["n_orphans"]) - int(r["n_assigned"])
                if i + 1 < i1:
                    n = carried[0] + ticks[i + 1]["n_new"]
                    g.launch_staged(10.0, n)
                    if i + 2 < len(ticks):
                        stage(ticks[i + 2])
                out.append(r)
            return out

        def start():
            g.load(st)
            g.set_eager_commit(not args.no_eager)  # every tick is waited for and committed
            carried[0] = 0
            torch.cuda.synchronize()
            stage(ticks[0])

        if mode == "hbm" and not args.no_pcie_pass:
            # the PCIe-inclusive rate (pinned host batches copied inside the timed region),
            # measured first on the same ticks from the same initial state: reported beside
            # the value, never as it
            mode = "pinned"
            prep(mode)
            start()
            loop(0, Wu)
            g.sync()
            t0 = time.perf_counter()
            rs = loop(Wu, Wu + K)
            g.sync()
            dtp = time.perf_counter() - t0
            na = sum(int(r["n_assigned"]) for r in rs)
            pcie = {"value": na / dtp, "ms_per_step": dtp * 1e3 / K, "events_in": "pinned host memory, H2D copies "
                    "inside the timed region (tick i+1's overlapping tick i)"}
            for tk in ticks:
                tk.pop("pin", None)
            mode = "hbm"
        prep(mode)
        start()
    else:
        import torch
        from faasbal.sharded import ShardedBalancer
        g = ShardedBalancer(rank, world, W, cap, max_events=E, device=dev)
        g.load(st)
        mode = "pageable"

        def run(i):
            tk = ticks[i]
            n = carried[0] + tk["n_new"]
            g.launch(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
            with torch.cuda.stream(g.stream):
                dist.all_reduce(g.exchange(), async_op=True).wait()  # phase 2 ordered after it on g.stream
            g.cont()
            r = g.wait()
            g.commit()
            carried[0] = n + int(r["n_orphans"]) - int(r["n_assigned"])
            return r

        def loop(i0, i1):
            return [run(i) for i in range(i0, i1)]

    def barrier():
        if dist is not None:
            t = torch.zeros(1, device="cuda")
            dist.all_reduce(t)
            torch.cuda.synchronize()

    loop(0, Wu)
    g.sync()
    barrier()
    g.sync()
    t0 = time.perf_counter()
    rs = loop(Wu, Wu + K)
    g.sync()
    barrier()
    dt = time.perf_counter() - t0
    B_ticks = 0  # SURVEY.md 8(d) bytes of the timed ticks (the log pass only on ticks with a death)
    for i, r in zip(range(Wu, Wu + K), rs):
        Ni, Oi = int(r["n_assigned"]), int(r["n_orphans"])
        Fi = int(r["log_head"]) - Ni if (Oi or int(r["n_evicted"])) else 0
        B_ticks += tick_bytes(W // world, 0, Fi // world, Oi, Ni, len(ticks[i]["ev_kind"]))
        stats["assigned"] += int(r["n_assigned"])
        stats["orphans"] += int(r["n_orphans"])
        stats["evicted"] += int(r["n_evicted"])  # sharded: this rank's evictions (summed below)
        stats["events"] += len(ticks[i]["ev_kind"])
    if dist is not None:
        t = torch.tensor([dt, float(stats["evicted"])], device="cuda", dtype=torch.float64)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:])
        dt, stats["evicted"] = float(t[0].item()), int(t[1].item())
    g.timing_enable(True)
    loop(Wu + K, len(ticks))
    kt = g.timing_read()
    g.timing_enable(False)
    wstats = g.window_stats() if world == 1 else (0, 0)
    kern = {k: ms / max(n, 1) * 1e3 for k, (ms, n) in kt.items()}  # us per launch
    per_tick = {k: ms / K * 1e3 for k, (ms, n) in kt.items()}      # us per tick
    line = {
        "metric": "streaming task assignments/sec, configs[4] (64K tasks + churn per tick, 1M workers)",
        "value": stats["assigned"] / dt,
        "unit": "assignments/s",
        "n_gpus": world,
        "steps": K,
        "warmup": Wu,
        "ms_per_step": dt * 1e3 / K,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (faasbal.synth.zipf_state(W, seed=0, dead_frac=0) + stream_ticks(seed=2))",
        "config": {"workload": "configs[4]: %d workers%s, %d new tasks + %d results + %d joins + %d heartbeats "
                               "per tick, %s, committed ticks"
                               % (W, "" if world == 1 else " sharded by worker-id range over %d GPUs" % world, T, T,
                                  0 if args.stream_quiet else max(1, W // 1000), max(1, int(args.hb_frac * W)),
                                  "a clock that ages nobody (no churn)" if args.stream_quiet else "10 ms per tick"),
                   "workers": W, "tasks_per_tick": T, "events_per_tick": stats["events"] / K,
                   "assigned_per_tick": stats["assigned"] / K,
                   "events_in": {"hbm": "HBM-resident (every tick's batch copied to the GPU before the timed "
                                         "region; read in place, checked by the tick's first kernel)",
                                  "pinned": "pinned host memory (H2D copies inside the timed region)",
                                  "pageable": "pageable (staged by copy)"}[mode],
                   "orphans_per_tick": stats["orphans"] / K, "evicted_per_tick": stats["evicted"] / K,
                   "parallelism": "dp1" if world == 1 else "worker-table shards x%d" % world},
        "tick": {"device_us_per_tick": sum(per_tick.values()), "kernels_us_per_tick": per_tick,
                 "kernels_us_per_launch": kern},
    }
    # roofline: the dominant kernel's share of SURVEY.md 8(d)'s tick bytes (one GPU: the apply
    # launch carries the slot purge, 24 B per worker, and the messages, 17 B each) over its
    # event-timed launch average; tick_frac: the whole tick's 8(d) bytes on the driver's clock
    # (by time per tick: a kernel of the occasional general tick -- k_scan, ~22 us once in
    # ~17 ticks -- may take longer per launch than the apply that runs every tick)
    dom = max(per_tick, key=lambda k: per_tick[k])
    Eavg = stats["events"] / K
    dom_bytes = (24 * W // world + 17 * Eavg) if dom == "ev_apply" else None
    traffic, traffic_src = None, None
    tp = os.path.join(REPO, "profiles", "traffic.json")
    if os.path.exists(tp):
        tj = json.load(open(tp)).get("entries", {}).get("stream,%d,%d,%d" % (W, T, world))
        # (timer names -> the kernel symbols the PMC summary keys: the window tick's emit is
        # k_emit_win, its apply k_ev_apply_ll)
        dk = {"ev_apply": "ev_apply_ll", "emit": "emit_win"}.get(dom, dom)
        if tj and dk in tj["kernels"]:
            traffic = tj["kernels"][dk]["hbm_bytes"]
            traffic_src = ("profiles/%s_pmc.csv (2*FETCH_SIZE + WRITE_SIZE per launch, separate rocprofv3 --pmc "
                           "passes; the x2 FETCH_SIZE correction is calibrated for streaming reads, so for random "
                           "gathers it is an upper bound)" % tj["tag"])
    ach = dom_bytes / (kern[dom] * 1e-6) / 1e9 if dom_bytes else None
    line["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS if ach else None, "traffic": traffic, "traffic_source": traffic_src,
                        "algorithmic_bytes": dom_bytes,
                        "bytes_model": "SURVEY.md 8(d) share: 24 W (the purge's 16 B read + 8 B write per worker) "
                                       "+ 17 E (messages)",
                        "kernel_avg_ms": kern[dom] * 1e-3,
                        "tick_bytes": B_ticks / K,
                        "tick_frac": B_ticks / dt / 1e9 / HBM_PEAK_GBS}
    if pcie is not None:
        line["pcie_inclusive"] = pcie
    if world == 1:
        # window ticks among all the ticks this process ran, and fallbacks
        line["tick"]["window_ticks"], line["tick"]["window_fallbacks"] = wstats
    if dist is not None:
        line["config"]["world_size_reported"] = dist.get_world_size()
        line["config"]["backend"] = dist.get_backend()
    if rank == 0:
        print(json.dumps(line), flush=True)


# The reference loop itself (task_dispatcher.py:324-419, CPython, one core), measured
# in the survey container with stub zmq/redis and a frozen clock: not
# re-run on the GPU box (the reference does not travel), carried for comparison.
REFERENCE_PYTHON = {"value": 82.7, "unit": "assignments/s", "cores": 1,
                    "sample": "SURVEY.md §6: reference start_heartbeat loop as written, W=64K, T=2K, Zipf free, "
                              "5% dead, measured in the survey container (CPython 3.10, stub I/O)",
                    "purge_once_value": 141816.0}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args):
    """`--gpus N` without a torch.distributed launcher around us: start the N rank
    processes (one per GPU) as children before anything touches the GPU, and exit
    with their status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def host_observed(g, st, T, steps, n_assigned):
    """Decisions the Python host can act on, on the path the drop-in dispatcher uses
    (GpuPushDispatcher._run -> GpuBalancer.tick(compact=True), dispatcher.py): per tick
    launch, wait, the per-message status bytes and the compact assignments -- slot and
    min(c, L + 1) per LRU position, written by the tick itself into registered pinned
    arrays, 5 B per queued worker -- with the orphans and evicted slots.  The dispatcher
    expands the compact form round by round while it sends (CompactAssignments); the
    whole expansion is timed beside it.  The tick is relaunched uncommitted (same
    workload every step); the commit (one kernel, then the host's bookkeeping) is timed
    separately and added per tick.  The per-task readback (4 B per task into pinned
    arrays, the dispatcher's path until round 5) is timed beside it too."""

    def timed(step):
        for _ in range(3):
            step()
        g.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        return (time.perf_counter() - t0) / steps

    def compact_path():
        out = g.tick(1000.0, 10.0, n_pending=T, commit=False, compact=True, pinned=True)
        assert len(out["assign"]) == n_assigned

    def per_task_path():
        out = g.tick(1000.0, 10.0, n_pending=T, commit=False, pinned=True)
        assert len(out["assign"]) == n_assigned

    dt_c = timed(compact_path)
    # the whole expansion of one tick's compact form (what the dispatcher's send loop walks)
    out = g.tick(1000.0, 10.0, n_pending=T, commit=False, compact=True, pinned=True)
    ca = out["assign"]
    te = time.perf_counter()
    for _ in range(5):
        full = ca.array()
    t_exp = (time.perf_counter() - te) / 5
    ref = g.tick(1000.0, 10.0, n_pending=T, commit=False, pinned=True)["assign"]
    if not np.array_equal(full, ref[:n_assigned]):
        raise SystemExit("host_observed: the expanded compact form differs from the per-task readback")
    g.set_compact(False)
    dt_t = timed(per_task_path)
    # the commit (one kernel + host bookkeeping), averaged over a few ticks, the
    # state reloaded (untimed) after each so every commit is the same tick's
    tc, nc = 0.0, 5
    for _ in range(nc):
        g.launch(1000.0, 10.0, n_pending=T)
        g.wait()
        t1 = time.perf_counter()
        g.commit()
        g.sync()
        tc += time.perf_counter() - t1
        g.load(st)
    tc /= nc
    Q = len(st["queue"])
    return {"value": n_assigned / (dt_c + tc), "unit": "assignments/s", "ms_per_tick": (dt_c + tc) * 1e3,
            "readback_ms_per_tick": dt_c * 1e3, "commit_ms": tc * 1e3, "readback_bytes": 5 * Q,
            "readback_form": "compact, the dispatcher's path: GpuBalancer.tick(compact=True) -- status bytes + slot "
                             "and min(c, L+1) per LRU position written by the tick into registered pinned arrays, "
                             "orphans / evicted in the same readback",
            "expand_ms": t_exp * 1e3, "value_with_expand": n_assigned / (dt_c + tc + t_exp),
            "per_task": {"value": n_assigned / (dt_t + tc), "ms_per_tick": (dt_t + tc) * 1e3,
                         "readback_bytes": 4 * n_assigned,
                         "form": "GpuBalancer.tick(pinned=True): slot per task into reusable pinned arrays"},
            "note": "launch + wait + readback of the tick's decisions (uncommitted relaunch), plus the commit "
                    "(average of 5); the dispatcher expands the compact form round by round as it sends "
                    "(faasbal.balancer.CompactAssignments), value_with_expand adds the whole expansion in numpy"}


def gated_timing(g, step, K, batch=64):
    """Per-kernel device times of K steps run back to back on the device: each batch of
    launches is queued behind a timing gate (fb_timing_gate) and released at once, so the
    host's enqueue pace cannot stretch them, and the packet events of every launch
    bracket that kernel's execution (the interval rocprofv3's kernel trace reports).  The
    kernels of one stream never overlap, so their sum per step cannot exceed the gated
    span per step (the gate's end to the release point's event), returned beside them."""
    g.timing_enable(True)
    span, done, timed_out = 0.0, 0, False
    while done < K:
        n = min(batch, K - done)
        g.timing_gate(True)
        for _ in range(n):
            step()
        g.timing_gate(False)
        ms, to = g.timing_span()
        span += ms
        timed_out |= to
        done += n
    kt = g.timing_read()
    g.timing_enable(False)
    return {k: (ms / n, n) for k, (ms, n) in kt.items()}, span / K, timed_out


def committed_tick(st, T, reps=5):
    """The tick with its commit.  A committed one-GPU tick defers its commit (the evicted
    records' deletion, task_dispatcher.py:246-247, and its orphans' log entries) into the
    next launch; after an idle tick that is k_scan's slot role (the records) and, on fused
    ticks, k_emit2's log workgroups (the log entries, tile by tile), else extra k_scan
    blocks -- so a stream of committed ticks has no commit launch of its own.  Measured on
    the tick after a committed tick (same state both times): its kernels with the folded
    commit, then relaunched uncommitted without it -- the difference is the commit's
    device cost inside the step.  The commit as its own kernel (what a state read in
    between forces) is timed beside it.  Packet-event device times of gated launches
    (gated_timing), averages of `reps`."""
    from faasbal import GpuBalancer
    g = GpuBalancer(len(st["reg"]), 2 * len(st["log"]) + 2 * T + 16, max_events=1, device=0)
    d_fold, d_plain, d_sep = [], [], []

    def step():
        g.launch(1000.0, 10.0, n_pending=T)

    for _ in range(reps):
        g.load(st)
        g.launch(1000.0, 10.0, n_pending=T)
        g.wait()
        g.commit()  # deferred: the next launch runs it
        k1, _, _ = gated_timing(g, step, 1)  # with the folded commit
        g.wait()
        k2, _, _ = gated_timing(g, step, 1)  # same tick, nothing left to fold
        g.wait()
        if not set(k2) <= set(k1):
            raise SystemExit("committed_tick: different kernels with and without the commit (%s / %s)"
                             % (sorted(k1), sorted(k2)))
        d_fold.append({k: v[0] for k, v in k1.items()})
        d_plain.append({k: v[0] for k, v in k2.items()})
        # the same commit as its own launch
        g.load(st)
        g.launch(1000.0, 10.0, n_pending=T)
        g.wait()
        g.commit()
        g.timing_enable(True)
        g.sync()  # flushes the deferred commit as its own kernel
        k3 = g.timing_read()
        g.timing_enable(False)
        d_sep.append(k3["commit"][0])
    g.close()
    f = {k: float(np.mean([d[k] for d in d_fold])) for k in d_fold[0]}
    p = {k: float(np.mean([d[k] for d in d_plain])) for k in d_plain[0]}
    # folded: no commit launch of its own (else the delta includes that launch)
    return dict(folded="commit" not in f, kernels_with_commit_ms=f, kernels_ms=p,
                commit_in_tick_ms=sum(f.values()) - sum(p.values()), commit_kernel_ms=float(np.mean(d_sep)),
                launches_per_committed_tick=len(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workers", type=int, default=65536)
    ap.add_argument("--tasks", type=int, default=1_000_000)
    ap.add_argument("--loads", default="zipf", choices=("zipf", "uniform"),
                    help="uniform: BASELINE configs[1]'s state (capacity 256, busy ~U[0,128); "
                         "use with --workers 1000 --tasks 100000)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-observed", action="store_true", help="skip the launch+wait+readback+commit timing")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--mode", default="heartbeat", choices=("heartbeat", "deque"),
                    help="deque: the loop without heartbeats (PushDispatcher.start), one GPU")
    ap.add_argument("--workload", default="tick", choices=("tick", "weak", "cfg3", "stream"),
                    help="tick: configs[2], 1M tasks x 64K workers (N GPUs: the same global table sharded N ways, "
                         "strong scaling); weak: N x 64K workers and N x 1M tasks sharded N ways; cfg3: configs[3], "
                         "16M tasks x 1M workers (N GPUs: the same global table sharded, strong scaling); stream: "
                         "configs[4], committed ticks with churn and 64K results each against 1M workers")
    ap.add_argument("--events", choices=("hbm", "pinned", "pageable"), default="hbm",
                    help="stream workload, one GPU: where each tick's message batch is when its tick starts")
    ap.add_argument("--no-eager", action="store_true",
                    help="stream workload: commit window ticks after the wait, not eagerly on the device")
    ap.add_argument("--no-pcie-pass", action="store_true",
                    help="stream workload: skip the PCIe-inclusive (pinned batches) pass beside the value")
    ap.add_argument("--pageable-events", action="store_true",
                    help="stream: messages in pageable numpy arrays (staging copies them into pinned memory)")
    ap.add_argument("--stream-quiet", action="store_true",
                    help="stream workload without churn: no re-registrations, no expiry (nobody dies)")
    ap.add_argument("--hb-frac", type=float, default=0.01,
                    help="stream: heartbeats per tick as a fraction of the workers (1.0: a 1M-message storm)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    if args.workload == "stream" and args.gpus == 1:
        return bench_stream(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but the launcher started %d ranks" % (args.gpus, world))
    dist = None
    dev = 0
    if world > 1:
        import torch
        import torch.distributed as dist
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        # the communication libraries print connection banners on stdout (gloo: "Rank 0 is
        # connected to ..."); keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(args.backend, device_id=torch.device("cuda", dev) if args.backend == "nccl" else None)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        if dist.get_world_size() != args.gpus:
            raise SystemExit("torch.distributed reports %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))
    if args.workload == "stream":
        bench_stream(args, dist, world, rank, dev)
        if dist is not None:
            dist.destroy_process_group()
        return

    from faasbal import GpuBalancer, synth

    # configs[2] (the metric's config): ONE global table of 64K workers and 1M pending
    # tasks, sharded by worker-id range over the N GPUs (strong scaling), the two-phase
    # tick with the RCCL exchange all-reduce every step; --workload weak:
    # N x 64K workers / N x 1M tasks (the pool grows with the GPUs)
    if args.workload == "cfg3":
        # configs[3]: one global table of 1M workers and 16M pending tasks, whatever N
        W = args.workers if args.workers != 65536 else 1 << 20
        T = args.tasks if args.tasks != 1_000_000 else 16_000_000
    elif args.workload == "weak":
        W, T = args.workers * world, args.tasks * world
    else:
        W, T = args.workers, args.tasks
    deque = args.mode == "deque"
    if deque and world > 1:
        raise SystemExit("--mode deque runs on one GPU (the start() loop has no sharded form)")
    # deque: same loads without deaths; 2 % of the queued workers hold a second deque entry
    if deque:
        st = synth.zipf_deque_state(W=W, seed=0, dup_frac=0.02)
    elif args.loads == "uniform":
        st = synth.uniform_state(W=W, seed=0)
    else:
        st = synth.zipf_state(W=W, seed=0)
    F = len(st["log"])
    Q = len(st["queue"])
    if world == 1:
        g = GpuBalancer(W, 2 * F + T + 16, max_events=1, device=0, mode=args.mode)
        g.load(st)

        def step():
            g.launch(1000.0, 10.0, n_pending=T)
    else:
        from faasbal.sharded import ShardedBalancer
        g = ShardedBalancer(rank, world, W, 2 * F + T + 16, max_events=1, device=dev)
        g.load(st)
        # the balancer's stream is torch's current stream for the whole run: the exchange
        # all-reduce is enqueued on it (phase 2 ordered after it, no host sync) without a
        # stream switch per step
        torch.cuda.set_stream(g.stream)

        def step():
            g.launch(1000.0, 10.0, n_pending=T)
            dist.all_reduce(g.exchange())
            g.cont()
    step()
    res = g.wait()
    n_assigned = int(res["n_assigned"])
    O = int(res["n_orphans"])
    n_evicted = int(res["n_evicted"])  # sharded: this rank's evicted slots; summed below
    if world > 1:
        t = torch.tensor([n_evicted], device="cuda", dtype=torch.int64)
        dist.all_reduce(t)
        n_evicted = int(t.item())

    def barrier():
        if dist is not None:
            t = torch.zeros(1, device="cuda")
            dist.all_reduce(t)
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    if world == 1:
        g.timing_mark()  # kernel traces: the timed region starts after this launch (tools/prof_summary.py)
    g.sync()
    # timed region: K back-to-back ticks on the device stream
    barrier()
    g.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_enq = time.perf_counter() - t0  # host enqueue of the K ticks (device still running)
    g.sync()
    barrier()
    dt = time.perf_counter() - t0
    if world == 1:
        g.timing_mark()  # ... and ends before this one
    if dist is not None:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # per-kernel device time with HIP packet events on the balancer's stream (same K): one
    # GPU, the K steps gated (run back to back on the device, gated_timing); sharded, the
    # exchange between the phases syncs with the host (gloo), so those launches are not gated
    gated_span_ms, gate_timed_out = None, False
    if world == 1:
        kern, gated_span_ms, gate_timed_out = gated_timing(g, step, args.steps)
        g.timing_mark()  # kernel traces: the gated pass (from its gate launch) ends before this one
    else:
        g.timing_enable(True)
        for _ in range(args.steps):
            step()
        kern = {k: (ms / n, n) for k, (ms, n) in g.timing_read().items()}
        g.timing_enable(False)
    g.wait()
    if world > 1:
        # the exchange: all-reduce time per tick, measured alone on the same stream
        xb = g.exchange()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(g.stream):
            for _ in range(5):
                dist.all_reduce(xb)
            barrier()
            ev0.record(g.stream)
            for _ in range(args.steps):
                dist.all_reduce(xb)
            ev1.record(g.stream)
        ev1.synchronize()
        kern["exchange_allreduce"] = (ev0.elapsed_time(ev1) / args.steps, args.steps)
        kt_x_bytes = xb.numel()

    # fused one-GPU heartbeat ticks (scan + emit only, W <= 128K slots): the emit's log
    # workgroups read the in-flight log and flag the orphans, k_scan has no log role
    log_in_emit = world == 1 and not deque and set(kern) == {"scan", "emit"} and W <= 1 << 17
    dom = max((k for k in kern if k != "exchange_allreduce"), key=lambda k: kern[k][0])
    dom_ms = kern[dom][0]
    tick_dev_ms = sum(v[0] for k, v in kern.items() if k != "exchange_allreduce")
    if dom == "emit" and deque:
        dom_bytes = emit_deque_bytes(Q, n_assigned, int(res["queue_len"]))
    elif dom == "emit" and world == 1:
        dom_bytes = emit_bytes(W, Q, F, O, n_assigned, int(res["queue_len"]), int(res["n_evicted"]),
                               log_in_emit=log_in_emit)
    elif dom == "emit":
        dom_bytes = emit_shard_bytes(Q, Q // world, F // world, int(res["n_orphans_local"]), int(res["n_local"]),
                                     int(res["queue_len"]))
    elif dom == "scan" and world == 1:
        dom_bytes = scan_bytes(W, Q, F, logscan="logscan" in kern or log_in_emit)
    elif dom == "logscan":
        dom_bytes = logscan_bytes(W, F)
    else:
        dom_bytes = tick_bytes(W // world, Q, F // world, O // world, n_assigned // world)
    B = tick_bytes(W, Q, F, O, n_assigned)
    # roofline bytes: SURVEY.md §8(d) -- the dominant kernel's share of the tick's bytes
    # (one-GPU configs[2]: the emit carries everything but k_scan's 16 B per worker read);
    # the builder's per-kernel model (queue / record traffic §8(d) does not count) beside it
    model_frac = dom_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    bytes_model = "SURVEY.md 8(d)"
    if dom == "emit" and world == 1 and not deque and set(kern) == {"scan", "emit"}:
        dom_bytes = B - 16 * W
        bytes_model = "SURVEY.md 8(d): tick bytes 24W + 4(N-O) + 4F + 8O minus k_scan's 16W read"
    else:
        bytes_model = "builder model (bench.py: %s_bytes)" % dom
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    value = n_assigned * args.steps / dt  # whole job: the global tick's dispatches
    # HBM bytes per launch of the dominant kernel from the committed PMC passes of
    # this same command (tools_profile.sh -> tools/prof_summary.py), when they match
    traffic, traffic_src, rocprof_ms = None, None, None
    tp = os.path.join(REPO, "profiles", "traffic.json")
    if os.path.exists(tp):
        tj = json.load(open(tp)).get("entries", {}).get("%d,%d,%d" % (W, T, world))
        if tj and dom in tj["kernels"]:
            traffic = tj["kernels"][dom]["hbm_bytes"]
            kd = tj["kernels"][dom]
            # the profile's gated timing pass (the regime kernel_avg_ms is measured in; cut at
            # bench.py's gate launches), else all launches
            rocprof_ms = (kd.get("trace_gated_avg_ns") or kd.get("trace_avg_ns") or 0) * 1e-6 or None
            traffic_src = ("profiles/%s_pmc.csv (2*FETCH_SIZE + WRITE_SIZE per launch, separate rocprofv3 --pmc "
                           "passes; the x2 FETCH_SIZE correction is calibrated for 16-B-per-lane streaming reads, "
                           "so for this kernel's 4-8 B gathers the figure is an upper bound), rocprof average over the "
                           "gated timing pass from profiles/%s_kernel_timed.csv (all launches: %s_kernel_stats.csv); "
                           "summary profiles/%s_traffic.json" % (tj["tag"], tj["tag"], tj["tag"], tj["tag"]))
    line = {
        "metric": "task assignments/sec + % HBM roofline, 1M tasks x 64K workers, 1/2/4/8 GPU",
        "value": value,
        "unit": "assignments/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "host_enqueue_ms_per_step": t_enq * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak" if args.workload == "weak" else "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (faasbal.synth.%s, seed=0)" % ("uniform_state" if args.loads == "uniform" else "zipf_state"),
        "config": {"workload": ("configs[3]: one tick, %d pending tasks x %d workers, Zipf(1.5) loads cap 32, 5%% "
                                "dead -> %d orphans redistributed, %s" % (
                                    T, W, O, "one GPU" if world == 1 else
                                    "worker table sharded by worker-id range over %d GPUs, exchange all-reduce of %d B "
                                    "per tick (%s)" % (world, kt_x_bytes, "RCCL" if args.backend == "nccl"
                                                       else args.backend))) if args.workload == "cfg3" else
                               ("configs[2] loads, start() loop (no heartbeats): one tick, %d pending tasks x %d "
                                "workers, Zipf(1.5) loads cap 32, deque of %d entries (2%% repeated ids)"
                                % (T, W, Q)) if deque else
                               ("configs[1]-style: one tick, %d pending tasks x %d workers, uniform loads (capacity "
                                "256, busy ~U[0,128)), %d orphans redistributed" % (T, W, O)) if args.loads == "uniform" else
                               ("configs[2]: one tick, %d pending tasks x %d workers, Zipf(1.5) loads cap 32, "
                                "5%% dead -> %d orphans redistributed" % (T, W, O)) if world == 1 else
                               ("configs[2]%s: one global tick of %d tasks x %d workers sharded by worker-id range "
                                "over %d GPUs, exchange all-reduce of %d B per tick (%s), %d orphans redistributed"
                                % (" per GPU (weak)" if args.workload == "weak" else "", T, W, world, kt_x_bytes,
                                   "RCCL" if args.backend == "nccl" else args.backend, O)),
                   "tasks_per_tick": T, "workers": W, "in_flight": F, "queue": Q,
                   "assigned_per_tick": n_assigned, "evicted": n_evicted,
                   "fill_level": int(res["fill_level"]),
                   "parallelism": "dp1" if world == 1 else "worker-table shards x%d" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes": dom_bytes, "bytes_model": bytes_model,
                     "kernel_avg_ms": dom_ms, "kernel_avg_ms_rocprof": rocprof_ms,
                     "frac_rocprof": (dom_bytes / (rocprof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if rocprof_ms else None,
                     "model_frac": model_frac,
                     # the whole tick on the driver's clock: SURVEY.md 8(d) tick bytes / ms_per_step
                     "tick_frac": B / (dt / args.steps) / 1e9 / HBM_PEAK_GBS},
        "tick": {"algorithmic_bytes": B, "device_ms": tick_dev_ms,
                 "achieved_GBs": B / (tick_dev_ms * 1e-3) / 1e9,
                 "kernels_avg_ms": {k: v[0] for k, v in kern.items()},
                 "kernel_timing": ("packet events of the K steps relaunched behind a timing gate (back to back on the "
                                   "device, bench.py: gated_timing)" if world == 1 else
                                   "packet events of K host-paced steps (the exchange syncs with the host)"),
                 "gate_timed_out": gate_timed_out},
    }
    # the per-kernel times must fit in the step they were measured for: their sum per step
    # against the timed region's ms_per_step.  (The gated span itself is not a step time: the
    # packet events add ~8 us between launches, profiles/r06b_trace_gaps.txt.)
    lim = dt * 1e3 / args.steps * 1.05
    line["tick"]["kernels_fit_step"] = bool(tick_dev_ms <= lim) and not gate_timed_out
    if not line["tick"]["kernels_fit_step"]:
        line["roofline"]["flag"] = ("per-kernel times (sum %.4f ms) exceed the step (%.4f ms x 1.05) or the gate timed "
                                    "out: roofline.frac is not a kernel property on this run" % (tick_dev_ms, lim / 1.05))
    if deque:
        line["metric"] = "task assignments/sec, start() loop (no heartbeats), 1M tasks x 64K workers"
        line["data"] = "synthetic (faasbal.synth.zipf_deque_state, seed=0, dup_frac=0.02)"
    if world > 1:
        line["config"]["world_size_reported"] = dist.get_world_size()
        line["config"]["backend"] = dist.get_backend()
    if args.workload == "cfg3":
        line["metric"] = "task assignments/sec, 16M tasks x 1M workers, 1/2/4/8 GPU"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_deque(st, T, args.cpu_budget) if deque else \
            cpu_baseline(st, T, args.cpu_budget)
        if not deque:
            line["reference_python_value"] = REFERENCE_PYTHON
    if world == 1 and not deque:
        cm = committed_tick(st, T)
        cm["device_ms_with_commit"] = tick_dev_ms + cm["commit_in_tick_ms"]
        cm["ms_per_step_with_commit"] = dt * 1e3 / args.steps + cm["commit_in_tick_ms"]
        cm["value_with_commit"] = n_assigned / (cm["ms_per_step_with_commit"] * 1e-3)
        # the headline is the committed tick: value / ms_per_step carry the commit's device cost
        # (task_dispatcher.py:246-249); the timed region's own figures stay beside them
        line["uncommitted"] = {"value": value, "ms_per_step": dt * 1e3 / args.steps,
                               "note": "the K timed steps alone: the functional tick relaunched, its commit not run"}
        line["value"] = cm["value_with_commit"]
        line["ms_per_step"] = cm["ms_per_step_with_commit"]
        line["roofline"]["tick_frac"] = B / (cm["ms_per_step_with_commit"] * 1e-3) / 1e9 / HBM_PEAK_GBS
        cm["note"] = ("the tick's commit (its %d evicted records' deletion and its %d orphaned log entries) "
                      "folded into the NEXT tick (folded): the records in k_scan's W role, the log entries "
                      "by k_emit2's log workgroup of each tile (fused ticks) or extra k_scan blocks. That next tick "
                      "runs on the committed, depleted state (kernels_ms: fewer queued positions and tasks than the "
                      "timed step's tick.kernels_avg_ms), so only the delta carries over: commit_in_tick_ms = its "
                      "kernels with the fold pending - the same tick relaunched without it (same state); "
                      "ms_per_step_with_commit = the timed region's ms_per_step + that delta (the line's value and "
                      "ms_per_step)" % (n_evicted, O))
        line["committed"] = cm
    if world == 1 and not args.no_host_observed:
        line["host_observed"] = host_observed(g, st, T, min(args.steps, 50), n_assigned)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
