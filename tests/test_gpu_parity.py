"""HIP balancer (through the C ABI) vs the oracle and the reference goldens.

Bit-exact on every output: per-event reconnect flags, task -> slot
assignments, orphan sequence numbers, evicted slots and the post-tick state
(registered, free_processes, last_heartbeat, LRU queue order, in-flight log).
"""
import glob
import os

import numpy as np
import pytest

from faasbal import GpuBalancer, FaasbalError, synth
from faasbal.balancer import TEST_PATHS
from oracle import Oracle, fixture_expect, fixture_ticks

pytestmark = pytest.mark.gpu
GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if not os.path.basename(p).startswith("deque_"))  # start_heartbeat vectors


def _state(scen):
    return dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
                queue=scen["init_queue"], log=scen["init_log"])


def _pair(st, log_cap, max_events=4096, purge_mode=1):
    W = len(st["reg"])
    g = GpuBalancer(W, log_cap, max_events=max_events)
    g.load(st)
    o = Oracle(W, log_cap, purge_mode=purge_mode)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    return g, o


def _cmp_out(a, b, t):
    for k in ("reconnect", "assign", "orphans", "evicted"):
        np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))


def _cmp_state(g, o, t):
    sg, so = g.read_state(), o.export()
    np.testing.assert_array_equal(sg["reg"], so["reg"], err_msg="tick %d reg" % t)
    reg = so["reg"].astype(bool)
    np.testing.assert_array_equal(sg["free"][reg], so["free"][reg], err_msg="tick %d free" % t)
    np.testing.assert_array_equal(sg["hb"][reg], so["hb"][reg], err_msg="tick %d hb" % t)
    np.testing.assert_array_equal(sg["queue"], so["queue"], err_msg="tick %d queue" % t)
    np.testing.assert_array_equal(sg["log"], so["log"], err_msg="tick %d log" % t)
    # the per-slot in-flight counts (O of the fused tick) equal the log's live entries
    # (kept by contexts whose died bitmap fits the fused tick's LDS: <= 128K slots)
    if g.max_workers <= 1 << 17:
        live = so["log"][so["log"] >= 0]
        np.testing.assert_array_equal(g.inflight(), np.bincount(live, minlength=len(so["reg"])).astype(np.uint32),
                                      err_msg="tick %d in-flight counts" % t)


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_golden_replay(path):
    z = np.load(path)
    W = int(z["W"])
    cap = len(z["init_log"]) + len(z["exp_assign"]) + 16
    g = GpuBalancer(W, cap, max_events=max(1, int(np.diff(z["ev_off"]).max(initial=0))))
    g.load_state(z["init_reg"], z["init_free"], z["init_hb"], z["init_epoch"], z["init_queue"], z["init_log"])
    carried = 0
    for t, tk in enumerate(fixture_ticks(z)):
        exp = fixture_expect(z, t)
        n = carried + tk["n_new"]
        out = g.tick(tk["now"], float(z["tte"]), tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"],
                     tk["ev_seq"], n)
        _cmp_out(out, exp, t)
        st = g.read_state(with_log=False)
        np.testing.assert_array_equal(st["queue"], exp["post_queue"], err_msg="tick %d queue" % t)
        np.testing.assert_array_equal(st["reg"], exp["post_reg"], err_msg="tick %d reg" % t)
        reg = exp["post_reg"].astype(bool)
        np.testing.assert_array_equal(st["free"][reg], exp["post_free"][reg])
        np.testing.assert_array_equal(st["hb"][reg], exp["post_hb"][reg])
        carried = n + len(out["orphans"]) - len(out["assign"])


@pytest.mark.parametrize("seed", range(40))
def test_random_multitick_vs_oracle(seed):
    W = [5, 37, 300, 1000][seed % 4]
    scen = synth.random_scenario(1000 + seed, W=W, n_ticks=6, max_events=[20, 200, 2000][seed % 3],
                                 max_new=[50, 400, 3000][(seed // 3) % 3])
    g, o = _pair(_state(scen), len(scen["init_log"]) + 40000)
    carried = 0
    for t, tk in enumerate(scen["ticks"]):
        # resolve result events to in-flight sequence numbers of the sender
        log = o.export()["log"]
        seq = np.full(len(tk["ev_kind"]), -1, np.int64)
        for i in np.nonzero(tk["ev_kind"] == synth.EV_RESULT)[0]:
            mine = np.nonzero(log == tk["ev_slot"][i])[0]
            if len(mine) and tk["ev_pick"][i] % 5 != 4:
                seq[i] = mine[tk["ev_pick"][i] % len(mine)]
        n = carried + tk["n_new"]
        args = (tk["now"], scen["tte"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp_out(a, b, t)
        _cmp_state(g, o, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


@pytest.mark.parametrize("seed", range(16))
def test_random_results_any_entry_vs_oracle(seed):
    """Results naming any log entry -- another worker's, a completed or redistributed
    one, the same entry twice in a tick, before and after the sender's death and
    re-registration -- against the oracle; in-flight counts checked every tick (the
    log is read-only during a tick, the commit clears the completed entries)."""
    W = [7, 64, 500, 3000][seed % 4]
    scen = synth.random_scenario(5000 + seed, W=W, n_ticks=8, max_events=[40, 400, 3000][seed % 3],
                                 max_new=[60, 500, 4000][(seed // 3) % 3])
    g, o = _pair(_state(scen), len(scen["init_log"]) + 60000)
    rng = np.random.default_rng(seed)
    carried = 0
    for t, tk in enumerate(scen["ticks"]):
        head = o.export()["head"]
        log = o.export()["log"]
        E = len(tk["ev_kind"])
        seq = rng.integers(-1, max(head, 1), E).astype(np.int64)
        own = np.nonzero(tk["ev_kind"] == synth.EV_RESULT)[0]
        # half the results name one of the sender's own entries (often the same one twice)
        for i in own[: len(own) // 2]:
            mine = np.nonzero(log == tk["ev_slot"][i])[0]
            if len(mine):
                seq[i] = mine[rng.integers(0, min(len(mine), 2))]
        n = carried + tk["n_new"]
        args = (tk["now"], scen["tte"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp_out(a, b, t)
        _cmp_state(g, o, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


def _compact_matches(g, where):
    """The compact form (slot, min(c, L + 1) per LRU position) read back and expanded
    on the host equals the per-task assignments."""
    n = g.last["n_assigned"]
    cap = g.max_workers + 2 * g.max_events + 16
    slot, c = g.pinned(cap, np.int32), g.pinned(cap, np.uint8)
    slot, c, _, _ = g.outputs_compact(slot, c)
    np.testing.assert_array_equal(g.expand(slot, c), g.assignments(), err_msg=where)
    return n


@pytest.mark.parametrize("seed", range(12))
def test_compact_assignments_random_multitick(seed):
    W = [5, 37, 300, 1000][seed % 4]
    scen = synth.random_scenario(7000 + seed, W=W, n_ticks=5, max_events=[20, 200, 2000][seed % 3],
                                 max_new=[50, 400, 3000][(seed // 3) % 3])
    g, o = _pair(_state(scen), len(scen["init_log"]) + 40000)
    g.set_compact(True)
    carried = 0
    for t, tk in enumerate(scen["ticks"]):
        n = carried + tk["n_new"]
        args = (tk["now"], scen["tte"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        g.launch(*args)
        g.wait()
        _compact_matches(g, "seed %d tick %d" % (seed, t))
        g.commit()
        b = o.tick(*args)
        carried = n + len(b["orphans"]) - len(b["assign"])


def test_compact_assignments_config2():
    st = synth.zipf_state(W=65536, seed=0)
    T = 1_000_000
    g = GpuBalancer(65536, 2 * len(st["log"]) + T + 16, max_events=1)
    g.load(st)
    g.set_compact(True)
    g.launch(1000.0, 10.0, n_pending=T)
    r = g.wait()
    assert _compact_matches(g, "configs[2]") == r["n_assigned"] > 0


@pytest.mark.parametrize("shape", ["config2", "random"])
def test_compact_outputs_written_during_the_tick(shape):
    """fb_set_compact_out: the tick writes its compact form, orphans and evicted slots into
    registered pinned arrays while it runs; after the wait they equal the per-task
    readback (configs[2]: a fused tick), and outputs into other arrays copy them over."""
    if shape == "config2":
        st, T, E = synth.zipf_state(W=65536, seed=0), 1_000_000, 1
        ticks = [dict(now=1000.0, ev=((), (), (), (), None), n=T)] * 2
    else:
        scen = synth.random_scenario(7100, W=1000, n_ticks=4, max_events=200, max_new=3000)
        st, T, E = _state(scen), 3000, 256
        ticks = [dict(now=tk["now"], ev=(tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"]),
                      n=tk["n_new"]) for tk in scen["ticks"]]
    W = len(st["reg"])
    g = GpuBalancer(W, 3 * len(st["log"]) + 4 * T + 16, max_events=max(E, 256))
    g.load(st)
    o = Oracle(W, 3 * len(st["log"]) + 4 * T + 16)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    cap = W + 2 * g.max_events + 16
    bufs = (g.pinned(cap, np.int32), g.pinned(cap, np.uint8), g.pinned(3 * len(st["log"]) + 4 * T + 16, np.int64),
            g.pinned(W, np.int32))
    g.set_compact_out(*bufs)
    for t, tk in enumerate(ticks):
        g.launch(tk["now"], 10.0, *tk["ev"], tk["n"])
        r = g.wait()
        slot, c, orph, ev = g.outputs_compact(*bufs)
        # against the oracle (g.orphans() / g.evicted() copy these same registered arrays)
        b = o.tick(tk["now"], 10.0, *[x if x is not None else [] for x in tk["ev"][:4]],
                   tk["ev"][4] if tk["ev"][4] is not None else np.full(len(tk["ev"][0]), -1, np.int64), tk["n"])
        np.testing.assert_array_equal(g.expand(slot, c), b["assign"], err_msg="tick %d assign (oracle)" % t)
        np.testing.assert_array_equal(orph, b["orphans"], err_msg="tick %d orphans (oracle)" % t)
        np.testing.assert_array_equal(ev, b["evicted"], err_msg="tick %d evicted (oracle)" % t)
        np.testing.assert_array_equal(g.expand(slot, c), g.assignments(), err_msg="tick %d assign" % t)
        np.testing.assert_array_equal(orph, g.orphans(), err_msg="tick %d orphans" % t)
        np.testing.assert_array_equal(ev, g.evicted(), err_msg="tick %d evicted" % t)
        other = (g.pinned(cap, np.int32), g.pinned(cap, np.uint8), g.pinned(max(len(orph), 1), np.int64),
                 g.pinned(max(len(ev), 1), np.int32))
        s2, c2, o2, e2 = g.outputs_compact(*other)
        np.testing.assert_array_equal(s2, slot)
        np.testing.assert_array_equal(c2, c)
        np.testing.assert_array_equal(e2, ev)
        if shape == "config2" and t == 0:
            assert r["n_orphans"] > 0 and r["n_evicted"] > 0
        g.commit()
    g.close()


def _one_tick_full(st, T, now=1000.0, tte=10.0):
    cap = len(st["log"]) + T + len(st["log"]) + 16
    g, o = _pair(st, cap)
    a = g.tick(now, tte, n_pending=T)
    b = o.tick(now, tte, [], [], [], [], [], T)
    return g, o, a, b


def test_config2_full_size():
    """BASELINE configs[1]: 100K tasks x 1K workers, uniform loads."""
    st = synth.uniform_state(W=1000, seed=0)
    g, o, a, b = _one_tick_full(st, 100_000)
    assert a["result"]["n_assigned"] == 100_000
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)


def test_config3_full_size():
    """BASELINE configs[2] (the headline): 1M tasks x 64K workers, Zipf loads,
    5 % heartbeat timeouts, in-flight tasks of dead workers redistributed."""
    st = synth.zipf_state(W=65536, seed=0)
    g, o, a, b = _one_tick_full(st, 1_000_000)
    r = a["result"]
    assert r["n_orphans"] > 0 and r["n_evicted"] > 0
    assert r["n_assigned"] == 1_000_000 + r["n_orphans"]
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)
    # size-independent properties
    alive = np.asarray(o.export()["reg"], bool)
    assert alive[a["assign"]].all()
    assert not alive[a["evicted"]].any()


def test_config4_single_gpu_full_size():
    """BASELINE configs[3] workload on one GPU: 16M tasks x 1M workers."""
    st = synth.zipf_state(W=1 << 20, seed=1)
    g, o, a, b = _one_tick_full(st, 16_000_000)
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)


def test_churn_stream_vs_oracle():
    """Config-5 shape (64K workers, reduced rate): joins, expiries and results each tick."""
    st = synth.zipf_state(W=65536, seed=3)
    ticks = synth.churn_ticks(st, n_ticks=4, seed=2, tasks_per_tick=65536, join_frac=0.001,
                              expire_frac=0.001, results_per_tick=8192)
    g, o = _pair(st, len(st["log"]) + 4 * 65536 + 200_000, max_events=20000)
    carried = 0
    for t, tk in enumerate(ticks):
        log = o.export()["log"]
        order = np.argsort(log, kind="stable")
        sl = log[order]
        seq = np.full(len(tk["ev_kind"]), -1, np.int64)
        for i in np.nonzero(tk["ev_kind"] == synth.EV_RESULT)[0]:
            s = tk["ev_slot"][i]
            lo, hi = np.searchsorted(sl, s), np.searchsorted(sl, s, side="right")
            if hi > lo:
                seq[i] = order[lo + tk["ev_pick"][i] % (hi - lo)]
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp_out(a, b, t)
        _cmp_state(g, o, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


def test_outputs_in_one_sync_match_the_single_copies():
    """fb_get_outputs (three DMA transfers, one sync) into pinned buffers returns the
    same lists as fb_get_assignments / fb_get_orphans / fb_get_evicted."""
    st = synth.zipf_state(W=4096, seed=3)
    g = GpuBalancer(4096, 2 * len(st["log"]) + 60000)
    g.load(st)
    g.launch(1000.0, 10.0, n_pending=50000)
    r = g.wait()
    a = g.pinned(r["n_assigned"] + 3, np.int32)
    o = g.pinned(r["n_orphans_local"] + 3, np.int64)
    e = g.pinned(r["n_evicted"] + 3, np.int32)
    ga, go, ge = g.outputs(a, o, e)
    assert r["n_orphans"] > 0 and r["n_evicted"] > 0
    np.testing.assert_array_equal(ga, g.assignments())
    np.testing.assert_array_equal(go, g.orphans())
    np.testing.assert_array_equal(ge, g.evicted())
    assert g.outputs(None, o, None)[1] is not None


def test_relaunch_without_commit_is_identical():
    st = synth.zipf_state(W=4096, seed=5)
    g = GpuBalancer(4096, len(st["log"]) * 2 + 200_000)
    g.load(st)
    outs = []
    for _ in range(3):
        g.launch(1000.0, 10.0, n_pending=50_000)
        g.wait()
        outs.append((g.assignments(), g.orphans(), g.evicted()))
    for x in outs[1:]:
        for u, v in zip(outs[0], x):
            np.testing.assert_array_equal(u, v)


def test_timing_gate_keeps_results():
    """bench.py's measurement hooks change no result: ticks queued behind the timing gate
    (released at once), marker launches between them, and a committed tick whose deferred
    commit rides in the gated launch, all against the oracle."""
    st = synth.zipf_state(W=4096, seed=7)
    g, o = _pair(st, len(st["log"]) * 2 + 400_000)
    g.timing_mark()
    g.timing_enable(True)
    g.timing_gate(True)
    for _ in range(3):
        g.launch(1000.0, 10.0, n_pending=50_000)
    g.timing_gate(False)
    ms, timed_out = g.timing_span()
    kt = g.timing_read()
    g.timing_enable(False)
    assert not timed_out and ms > 0 and kt and all(n == 3 for _, n in kt.values())
    g.wait()
    b = o.tick(1000.0, 10.0, [], [], [], [], [], 50_000)
    _cmp_out(dict(reconnect=g.event_status(), assign=g.assignments(), orphans=g.orphans(), evicted=g.evicted()),
              b, 0)
    g.commit()  # deferred into the next (gated) launch
    g.timing_mark()
    g.timing_gate(True)
    g.launch(1001.0, 10.0, n_pending=20_000)
    g.timing_gate(False)
    g.wait()
    b = o.tick(1001.0, 10.0, [], [], [], [], [], 20_000)
    _cmp_out(dict(reconnect=g.event_status(), assign=g.assignments(), orphans=g.orphans(), evicted=g.evicted()),
              b, 1)
    g.commit()
    _cmp_state(g, o, 1)


def test_wide_free_counts_rerun():
    """A result pushes free past the launch's round table: the tick reruns wider."""
    W = 3
    st = dict(reg=np.ones(W, np.uint8), free=np.array([64, 3, 200], np.int32), hb=np.full(W, 999.0),
              epoch=np.zeros(W, np.uint32), queue=np.array([0, 1], np.int32), log=np.array([0, 0], np.int32))
    g, o = _pair(st, 10_000)
    args = (1000.0, 10.0, [synth.EV_RESULT], [0], [0], [999.5], [1], 1000)
    a, b = g.tick(*args), o.tick(*args)
    assert a["result"]["reruns"] >= 1
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)
    # large counts by register/reconnect
    args = (1001.0, 10.0, [synth.EV_REGISTER, synth.EV_RECONNECT], [2, 1], [3000, 7], [1000.5, 1000.7], [-1, -1],
            5000)
    a, b = g.tick(*args), o.tick(*args)
    _cmp_out(a, b, 1)
    _cmp_state(g, o, 1)


def test_edge_cases():
    # no workers registered, tasks pending
    st = dict(reg=np.zeros(4, np.uint8), free=np.zeros(4, np.int32), hb=np.zeros(4), epoch=np.zeros(4, np.uint32),
              queue=np.zeros(0, np.int32), log=np.zeros(0, np.int32))
    g, o = _pair(st, 1000)
    for t, args in enumerate([
        (10.0, 10.0, [], [], [], [], [], 5),                        # empty everything
        (11.0, 10.0, [synth.EV_HEARTBEAT], [2], [0], [10.5], [-1], 5),  # unknown id -> reconnect
        (12.0, 10.0, [synth.EV_RESULT], [2], [0], [11.0], [-1], 5),     # free 0 -> 1: back of queue
        (40.0, 10.0, [], [], [], [], [], 5),                        # everybody expires
    ]):
        a, b = g.tick(*args), o.tick(*args)
        _cmp_out(a, b, t)
        _cmp_state(g, o, t)


def test_log_full_is_an_error():
    st = synth.uniform_state(W=100, seed=1)
    g = GpuBalancer(100, 1000)
    g.load(st)
    with pytest.raises(FaasbalError):
        g.tick(1000.0, 10.0, n_pending=5000)


@pytest.mark.parametrize("window,eager", [(0, 0), (1, 0), (1, 1)])
def test_device_reported_lengths_are_validated(window, eager):
    """fb_tick_wait checks every device-reported length against its buffer before any
    copy uses it: a queue length past the buffer (injected into the results) fails the
    tick with FB_EHIP naming the number; the tick is not committed and the next one runs
    against the oracle as if it never happened.  Eager window commits (enqueued behind the
    tick at launch): the device checks the window it reports with the same bounds, so the
    commit kernel commits nothing either."""
    # nobody dead and a frozen clock: both ticks stay at fill level 0, so with window ticks
    # on the second one is a window tick (a death's orphans would lift it to level 1: a
    # general tick after the window attempt)
    st = synth.zipf_state(W=2048, seed=3, dead_frac=0.0)
    g, o = _pair(st, len(st["log"]) * 2 + 100_000)
    g.set_window(window)
    g.set_eager_commit(bool(eager))
    args = (1000.0, 10.0, [], [], [], [], [], 500)
    a, b = g.tick(*args), o.tick(*args)
    _cmp_out(a, b, 0)
    g.set_path("fault_qlen", 1 << 30)
    args = (1000.0, 10.0, [synth.EV_HEARTBEAT], [5], [0], [1000.0], [-1], 300)
    with pytest.raises(FaasbalError, match="queue length|window"):
        g.tick(*args)
    a, b = g.tick(*args), o.tick(*args)
    _cmp_out(a, b, 1)
    _cmp_state(g, o, 1)
    assert g.window_stats()[0] == window


def test_invalid_events_rejected():
    st = synth.uniform_state(W=10, seed=1)
    g = GpuBalancer(10, 1000)
    g.load(st)
    with pytest.raises(FaasbalError):
        g.tick(1000.0, 10.0, [0], [10], [1], [999.0], [-1], 0)   # slot out of range
    with pytest.raises(FaasbalError):
        g.tick(1000.0, 10.0, [0, 0], [1, 2], [1, 1], [999.0, 998.0], [-1, -1], 0)  # ts decreasing


@pytest.mark.parametrize("bad", ["decreasing", "future", "slot", "kind"])
def test_invalid_messages_in_pinned_batches(bad):
    """Pinned message arrays are checked by k_ev_link, not read by the host: the tick
    fails at wait naming the first offending event, commits nothing (an out-of-range
    slot or unknown kind is neutralised before any use), and the next tick runs."""
    st = synth.uniform_state(W=64, seed=1)
    g, o = _pair(st, 4000)
    ts = np.array([999.0, 999.5, 998.0 if bad == "decreasing" else 999.6, 999.7])
    kinds = np.array([2, 2, 2, 2], np.uint8)
    slots = np.array([1, 2, 3, 4], np.int32)
    if bad == "future":
        ts[3] = 1000.5
    if bad == "slot":
        slots[2] = 1 << 20
    if bad == "kind":
        kinds[3] = 9
    k, s, v, t, q = g.pin_events(kinds, slots, np.zeros(4, np.int32), ts, np.full(4, -1, np.int64))
    with pytest.raises(FaasbalError, match="event %d" % (2 if bad in ("decreasing", "slot") else 3)):
        g.tick(1000.0, 10.0, k, s, v, t, q, 10)
    args = (1000.0, 10.0, np.array([2], np.uint8), np.array([5], np.int32), np.zeros(1, np.int32),
            np.array([999.0]), np.full(1, -1, np.int64), 10)
    a, b = g.tick(*args), o.tick(*args)
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)


@pytest.fixture
def force_plan(monkeypatch):
    """Route ticks through the 3-launch path (k_plan), used for large grids."""
    monkeypatch.setitem(TEST_PATHS, "plan", 1)


@pytest.mark.parametrize("seed", range(8))
def test_random_multitick_plan_path(force_plan, seed):
    test_random_multitick_vs_oracle(seed)


def test_config3_plan_path(force_plan):
    test_config3_full_size()


def test_golden_plan_path(force_plan):
    for path in GOLDEN[:12] + GOLDEN[-3:]:
        test_golden_replay(path)


@pytest.fixture
def force_chunked_emit(monkeypatch):
    """The 3-launch path with the chunked k_emit (used when R > 128) instead of
    k_emit2 after k_plan."""
    monkeypatch.setitem(TEST_PATHS, "plan", 2)


@pytest.mark.parametrize("seed", range(4))
def test_random_multitick_chunked_emit(force_chunked_emit, seed):
    test_random_multitick_vs_oracle(seed)


def test_config3_chunked_emit(force_chunked_emit):
    test_config3_full_size()


def test_device_primitives_selftest():
    g = GpuBalancer(16, 16)
    assert g.selftest() == 0


@pytest.fixture
def logscan(monkeypatch):
    """Route the log role through k_logscan (died bitmap in LDS), the default past 128K slots."""
    monkeypatch.setitem(TEST_PATHS, "logscan", 1)


@pytest.fixture
def split_slots(monkeypatch):
    """Separate k_slots launch + global died bitmap (tables too large for k_logscan's LDS)."""
    monkeypatch.setitem(TEST_PATHS, "logscan", 0)
    monkeypatch.setitem(TEST_PATHS, "split_slots", 1)


@pytest.mark.parametrize("seed", range(12))
def test_random_multitick_logscan(logscan, seed):
    test_random_multitick_vs_oracle(seed)


@pytest.mark.parametrize("seed", range(6))
def test_random_multitick_logscan_plan(logscan, force_plan, seed):
    """Large-table path with k_logscan: no k_plan2 (k_emit2 reduces the group rows, the last
    k_logscan workgroup writes the tile prefixes -- the configs[3] default)."""
    test_random_multitick_vs_oracle(seed + 20)


@pytest.mark.parametrize("seed", range(4))
def test_random_multitick_logscan_plan2(logscan, force_plan, monkeypatch, seed):
    """... and the same ticks through k_plan2 (fb_set_path("gp", 0))."""
    monkeypatch.setitem(TEST_PATHS, "gp", 0)
    test_random_multitick_vs_oracle(seed + 20)


def test_config3_logscan_plan2(logscan, force_plan, monkeypatch):
    monkeypatch.setitem(TEST_PATHS, "gp", 0)
    test_config3_full_size()


def test_config3_logscan(logscan):
    test_config3_full_size()


@pytest.mark.parametrize("wtiles", [1, 2])
@pytest.mark.parametrize("seed", range(2))
def test_random_multitick_logscan_plan_wtiles(logscan, force_plan, monkeypatch, seed, wtiles):
    """k_scan's slot purge with 1 or 2 tiles per W workgroup (fb_set_path("wtiles"); large
    tables default to 4, fused ones to 1)."""
    monkeypatch.setitem(TEST_PATHS, "wtiles", wtiles)
    test_random_multitick_vs_oracle(seed + 30)


@pytest.mark.parametrize("seed", range(3))
def test_random_multitick_logscan_plan_qtiles1(logscan, force_plan, monkeypatch, seed):
    """k_scan's queue role with one queue block per workgroup (fb_set_path("qtiles", 1));
    unfused one-GPU tables default to four per workgroup."""
    monkeypatch.setitem(TEST_PATHS, "qtiles", 1)
    test_random_multitick_vs_oracle(seed + 20)


@pytest.mark.parametrize("seed", range(3))
def test_random_multitick_logscan_plan_no_cmix(logscan, force_plan, monkeypatch, seed):
    """k_emit2's grid in role order (fb_set_path("cmix", 0)): queue blocks, then the
    compaction workgroups -- the default interleaves their rows."""
    monkeypatch.setitem(TEST_PATHS, "cmix", 0)
    test_random_multitick_vs_oracle(seed + 20)


def test_churn_logscan(logscan):
    test_churn_stream_vs_oracle()


def test_golden_logscan(logscan):
    for path in GOLDEN:
        test_golden_replay(path)


@pytest.mark.parametrize("seed", range(6))
def test_random_multitick_split_slots(split_slots, seed):
    test_random_multitick_vs_oracle(seed + 30)


def test_config4_split_slots(split_slots):
    test_config4_single_gpu_full_size()


def test_relaunch_with_other_messages_is_clean():
    """A launched-but-abandoned tick (no commit) must leave no marks: the next
    launch, with other messages, equals the oracle run without the first."""
    for seed in range(4):
        scen = synth.random_scenario(4100 + seed, W=300, n_ticks=3, max_events=300, max_new=500)
        g, o = _pair(_state(scen), len(scen["init_log"]) + 40000)
        carried = 0
        for t, tk in enumerate(scen["ticks"]):
            n = carried + tk["n_new"]
            # an abandoned launch with the events of a different slot mapping
            g.launch(tk["now"], scen["tte"], tk["ev_kind"], (tk["ev_slot"] * 7 + 3) % scen["W"], tk["ev_val"],
                     tk["ev_ts"], None, n)
            g.wait()
            args = (tk["now"], scen["tte"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"],
                    np.full(len(tk["ev_kind"]), -1, np.int64), n)
            a, b = g.tick(*args), o.tick(*args)
            _cmp_out(a, b, t)
            _cmp_state(g, o, t)
            carried = n + len(b["orphans"]) - len(b["assign"])


def test_stream_ticks_vs_oracle():
    """configs[4] event mix (results of in-flight tasks, joins, heartbeats,
    expiry by clock) at reduced size, committed ticks."""
    st = synth.zipf_state(W=8192, seed=0, dead_frac=0.0)
    ticks = synth.stream_ticks(st, n_ticks=6, seed=2, tasks_per_tick=4096, results_per_tick=4096, dt=1.5)
    g, o = _pair(st, len(st["log"]) + 6 * 8192 + 16, max_events=8192)
    carried = 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp_out(a, b, t)
        _cmp_state(g, o, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


@pytest.mark.parametrize("pinned", [False, True], ids=["copied", "zero-copy"])
def test_stream_ticks_staged_pipeline_vs_oracle(pinned):
    """fb_tick_stage of tick t+1 while tick t runs (double-buffered pinned staging),
    then fb_tick_launch_staged: the same outputs and states as the oracle.  Zero-copy:
    the messages already sit in pinned host memory (GpuBalancer.pin_events), staging
    validates them in place and the H2D copies read them (one tick's without seq)."""
    st = synth.zipf_state(W=8192, seed=0, dead_frac=0.0)
    ticks = synth.stream_ticks(st, n_ticks=6, seed=3, tasks_per_tick=4096, results_per_tick=4096, dt=1.5)
    g, o = _pair(st, len(st["log"]) + 6 * 8192 + 16, max_events=8192)
    if pinned:
        for i, tk in enumerate(ticks):
            (tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq) = g.pin_events(
                tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"])
            if i == 2:  # no sequence numbers: results of tasks the balancer never saw
                tk["ev_seq"] = None
            else:
                tk["ev_seq"] = seq

    def stage(tk):
        g.stage(tk["now"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"])

    carried = 0
    stage(ticks[0])
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        g.launch_staged(10.0, n)
        if t + 1 < len(ticks):
            stage(ticks[t + 1])  # host work overlapping the device tick
        g.wait()
        a = dict(reconnect=g.event_status(), assign=g.assignments(), orphans=g.orphans(), evicted=g.evicted())
        g.commit()
        seq = tk["ev_seq"] if tk["ev_seq"] is not None else np.full(len(tk["ev_kind"]), -1, np.int64)
        b = o.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        _cmp_out(a, b, t)
        _cmp_state(g, o, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


def test_launch_staged_needs_stage():
    st = synth.zipf_state(W=512, seed=1)
    g = GpuBalancer(512, len(st["log"]) * 2 + 4096)
    g.load(st)
    with pytest.raises(FaasbalError):
        g.launch_staged(10.0, 10)
    g.stage(1000.0)
    g.launch_staged(10.0, 100)
    g.wait()
    with pytest.raises(FaasbalError):  # a stage is consumed by its launch
        g.launch_staged(10.0, 100)


def _sort_tick(W, E, hot_frac, seed, purge_mode=1, hot_n=5, expect_reruns=None):
    """One tick of E messages (kinds mixed, clocks ascending) on a W-slot table,
    hot_frac of them on hot_n hot slots; GPU vs oracle.  The oracle purges after
    every message (purge_mode 1: O(W) each, so E * W stays around 1e9; 2: heap)."""
    rng = np.random.default_rng(seed)
    st = synth.zipf_state(W=W, seed=seed % 7, dead_frac=0.02)
    hot = rng.choice(W, size=hot_n, replace=False)
    slot = np.where(rng.random(E) < hot_frac, hot[rng.integers(0, hot_n, E)], rng.integers(0, W, E)).astype(np.int32)
    kind = rng.choice([synth.EV_REGISTER, synth.EV_HEARTBEAT, synth.EV_RESULT, synth.EV_RECONNECT], size=E,
                      p=[0.1, 0.4, 0.4, 0.1]).astype(np.int32)
    val = rng.integers(0, 4, E).astype(np.int32)
    now = 1000.0  # zipf_state's clock
    ts = np.sort(now - rng.random(E)).astype(np.float64)
    g, o = _pair(st, 2 * len(st["log"]) + 100_000, max_events=E, purge_mode=purge_mode)
    args = (now, 10.0, kind, slot, val, ts, np.full(E, -1, np.int64), 20_000)
    a, b = g.tick(*args), o.tick(*args)
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)
    if expect_reruns is not None and TEST_PATHS.get("ev_ll", 1) != 0:  # reruns: linked-list path only
        assert (a["result"]["reruns"] > 0) == expect_reruns, a["result"]["reruns"]


@pytest.fixture
def radix(monkeypatch):
    """fb_set_path("ev_ll", 0): every message tick groups its events by the radix sort."""
    monkeypatch.setitem(TEST_PATHS, "ev_ll", 0)


@pytest.mark.parametrize("W,E,wide", [((1 << 17) + 5, 12000, "1"), (1 << 20, 2000, "1"), (1 << 21, 1000, "1"),
                                      ((1 << 17) + 5, 12000, "0"), (1 << 20, 2000, "0")])
def test_event_sort_wide_digits(radix, monkeypatch, W, E, wide):
    """Slot spaces of 17-22 bits: the event sort runs two passes of 9-11-bit
    digits (fb_set_path("rs_wide", 0): three of 8 bits); identical to the oracle."""
    monkeypatch.setitem(TEST_PATHS, "rs_wide", int(wide))
    _sort_tick(W, E, 0.0, W + E)


@pytest.mark.parametrize("W,E", [(300, 30000), (5000, 30000), ((1 << 19) + 3, 2000)])
def test_event_sort_stable_on_repeated_slots(W, E):
    """90 % of the messages on five slots (equal-key runs across sort tiles): the
    per-slot arrival order the sort must keep decides every register / result.
    The linked-list grouping gives up on these slots (> 16 messages) and the tick
    reruns through the sort."""
    _sort_tick(W, E, 0.9, W, expect_reruns=True)


@pytest.mark.parametrize("W,E,hot_frac,hot_n", [((1 << 20), 77_000, 0.0, 5), (4096, 20_000, 0.0, 5),
                                                (1 << 17, 30_000, 0.02, 128), (1 << 17, 3_000, 0.05, 20)])
def test_event_link_grouping(W, E, hot_frac, hot_n):
    """The default grouping of a message tick on one GPU: per-slot linked lists
    (k_ev_link), each slot's messages (up to 16) sorted into arrival order in
    registers by k_ev_apply_ll -- no radix sort and no rerun; identical to the oracle.
    (4096 slots x 20 K messages: about 5 per slot, 0.2 % of slots with 13-16.)"""
    _sort_tick(W, E, hot_frac, W + E + 3, purge_mode=2, hot_n=hot_n, expect_reruns=False)


@pytest.mark.parametrize("n_hot", [16, 17])
def test_event_link_limit(n_hot):
    """Exactly 16 messages on one slot stay on the linked-list path; 17 rerun the
    tick through the sort.  Both identical to the oracle."""
    W, E = 1000, 600
    rng = np.random.default_rng(n_hot)
    st = synth.zipf_state(W=W, seed=3, dead_frac=0.02)
    slot = rng.permutation(np.concatenate([np.full(n_hot, 7), rng.choice(np.arange(8, W), E - n_hot,
                                                                          replace=False)])).astype(np.int32)
    kind = rng.choice([synth.EV_REGISTER, synth.EV_HEARTBEAT, synth.EV_RESULT, synth.EV_RECONNECT], size=E,
                      p=[0.1, 0.4, 0.4, 0.1]).astype(np.int32)
    val = rng.integers(0, 4, E).astype(np.int32)
    ts = np.sort(1000.0 - rng.random(E)).astype(np.float64)
    g, o = _pair(st, 2 * len(st["log"]) + 100_000, max_events=E)
    args = (1000.0, 10.0, kind, slot, val, ts, np.full(E, -1, np.int64), 3000)
    a, b = g.tick(*args), o.tick(*args)
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)
    if TEST_PATHS.get("ev_ll", 1) != 0:
        assert (a["result"]["reruns"] > 0) == (n_hot > 16)


@pytest.mark.parametrize("W,E,wide", [(1 << 20, 300_000, "1"), ((1 << 17) + 5, 1_200_000, "1"),
                                      ((1 << 17) + 5, 1_200_000, "0"), (1 << 20, 2_000_000, "1")])
def test_event_sort_large_batches(radix, monkeypatch, W, E, wide):
    """Batches of more than kRsScanMin sort tiles (E > 128 K): the column prefixes
    of the [tile][digit] counts come from their own launch (k_rs_scan) before each
    scatter; identical to the oracle (heap purge) up to 2 M messages in one tick."""
    monkeypatch.setitem(TEST_PATHS, "rs_wide", int(wide))
    _sort_tick(W, E, 0.3, W + E, purge_mode=2)


@pytest.mark.parametrize("W,dead", [(8192, 0.05), (65536, 0.05)])
def test_idle_ticks_commit_folded_into_scan(W, dead):
    """Committed idle ticks back to back (the configs[2] shape: no messages, a clock that
    advances so workers keep expiring): each tick's commit -- the evicted records'
    deletion (task_dispatcher.py:246-247) and its orphaned log entries -- rides in the
    next tick's k_scan (W role and extra blocks); outputs, state and in-flight counts
    equal the oracle's every tick, also when a state read flushes the commit first."""
    st = synth.zipf_state(W=W, seed=5, dead_frac=dead)
    T = 4 * W
    g, o = _pair(st, len(st["log"]) + 12 * T + 16)
    carried = 0
    for t in range(6):
        now = 1000.0 + 1.5 * t
        n = carried + T
        args = (now, 10.0, [], [], [], [], [], n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp_out(a, b, t)
        assert t > 0 or len(b["evicted"]) > 0
        if t % 2:  # a state read flushes the pending commit as its own launch
            _cmp_state(g, o, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    _cmp_state(g, o, 6)
    g.close()


@pytest.mark.parametrize("path", ["fused", "plan"])
@pytest.mark.parametrize("L", [0, 1, 30, 31, 32, 33, 62])
def test_fill_levels_around_table_widths(monkeypatch, path, L):
    """Fill levels either side of the 32 / 64-row round tables (a table is chosen from the
    largest free count, so L + 2 rows must fit), a partial round L, dead workers and their
    orphans dispatched first, on the fused and the k_plan paths, against the oracle."""
    if path == "plan":
        monkeypatch.setitem(TEST_PATHS, "plan", 1)
    W = 3000
    rng = np.random.default_rng(100 + L)
    free = rng.integers(L + 2, L + 40, W).astype(np.int32)  # every live worker has c > L + 1
    hb = np.where(rng.random(W) < 0.05, 900.0, 999.0)        # 5 % expire at now = 1000
    log = rng.integers(0, W, 4 * W).astype(np.int32)
    st = dict(reg=np.ones(W, np.uint8), free=free, hb=hb, epoch=np.zeros(W, np.uint32),
              queue=rng.permutation(W).astype(np.int32), log=log)
    g, o = _pair(st, len(log) + W * (L + 2) + 16)
    alive = int((hb > 990.0).sum())
    dead_inflight = int(np.isin(log, np.nonzero(hb < 990.0)[0]).sum())
    T = alive * L + alive // 3 - dead_inflight  # L full rounds, then a third of round L
    args = (1000.0, 10.0, [], [], [], [], [], max(T, 0))
    a, b = g.tick(*args), o.tick(*args)
    if T > 0:
        assert a["result"]["fill_level"] == L, a["result"]
    _cmp_out(a, b, 0)
    _cmp_state(g, o, 0)
