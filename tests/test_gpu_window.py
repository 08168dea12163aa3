"""Window ticks (the sliding level-0 queue) vs the oracle.

A level-0 tick serves a prefix of the LRU queue; as a window tick it leaves the rest
of the queue in place (positions whose slot left become tombstones) and appends the
re-queued workers at the tail.  Every output and the post-tick state must equal the
oracle's (task_dispatcher.py:324-419 restated) whichever path a tick takes, including
general ticks that read a window with tombstones and window ticks that fall back to
the general path.  Window mode is forced on small contexts (fb_set_window(1)); the
1M-worker stream of tests/test_full_size.py runs it in its default (auto) mode.
"""
import numpy as np
import pytest

from faasbal import GpuBalancer, FaasbalError, _lib, synth
from oracle import Oracle

pytestmark = pytest.mark.gpu


def _pair(st, log_cap, max_events, window=1, purge_mode=1, eager=False):
    W = len(st["reg"])
    g = GpuBalancer(W, log_cap, max_events=max_events)
    g.set_window(window)
    g.set_eager_commit(eager)
    g.load(st)
    o = Oracle(W, log_cap, purge_mode=purge_mode)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    return g, o


def _cmp(g, o, a, b, t):
    for k in ("reconnect", "assign", "orphans", "evicted"):
        np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))
    assert a["result"]["queue_len"] == len(o.export()["queue"]), "tick %d: queue length" % t
    sg, so = g.read_state(), o.export()
    np.testing.assert_array_equal(sg["reg"], so["reg"], err_msg="tick %d reg" % t)
    reg = so["reg"].astype(bool)
    np.testing.assert_array_equal(sg["free"][reg], so["free"][reg], err_msg="tick %d free" % t)
    np.testing.assert_array_equal(sg["hb"][reg], so["hb"][reg], err_msg="tick %d hb" % t)
    np.testing.assert_array_equal(sg["queue"], so["queue"], err_msg="tick %d queue" % t)
    np.testing.assert_array_equal(sg["log"], so["log"], err_msg="tick %d log" % t)


def _stream(seed, W, T, dt, n_ticks, hb_frac=0.01, join_frac=0.002):
    st = synth.zipf_state(W=W, seed=seed, dead_frac=0.0)
    ticks = synth.stream_ticks(st, n_ticks=n_ticks, seed=seed + 7, tasks_per_tick=T, results_per_tick=T,
                               dt=dt, hb_frac=hb_frac, join_frac=join_frac)
    return st, ticks


@pytest.mark.parametrize("eager", [False, True])
@pytest.mark.parametrize("seed,W,T,dt", [(0, 8192, 512, 0.5), (1, 8192, 1024, 0.6), (2, 4096, 256, 0.5),
                                         (3, 20000, 2048, 0.05), (4, 8192, 64, 0.3)])
def test_window_stream_vs_oracle(seed, W, T, dt, eager):
    """configs[4]'s event mix at reduced size: results of in-flight tasks, joins (moved
    to the front), heartbeats (kept in place, refreshed at commit), expiry by the clock
    (tombstones); most ticks run as window ticks.  eager: each window tick's commit is
    enqueued behind it at launch (fb_set_eager_commit)."""
    st, ticks = _stream(seed, W, T, dt, n_ticks=10)
    E = max(len(t["ev_kind"]) for t in ticks)
    g, o = _pair(st, 3 * len(st["log"]) + 20 * T + 16, max_events=E, purge_mode=2, eager=eager)
    carried = 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp(g, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    wt, fb = g.window_stats()
    assert wt >= 5, "window ticks: %d (fallbacks %d)" % (wt, fb)
    g.close()


@pytest.mark.parametrize("eager", [False, True])
@pytest.mark.parametrize("seed,W,T", [(0, 8192, 512), (1, 20000, 2048)])
def test_window_ticks_without_deaths(seed, W, T, eager):
    """Window ticks in which no registration dies (no re-registrations, a clock that does
    not age anyone) skip the log scan (k_logscan reads no entry: every tile count zero);
    every third tick the clock jumps 0.4 s (~4 % of the workers expire) and keeps its
    re-registrations, so its orphans are flagged.  Alternating the two checks that a
    stale death mark of an earlier launch never passes for this one."""
    st, ticks = _stream(seed, W, T, 0.0, n_ticks=12)
    E = max(len(t["ev_kind"]) for t in ticks)
    g, o = _pair(st, 3 * len(st["log"]) + 24 * T + 16, max_events=E, purge_mode=2, eager=eager)
    carried = 0
    n_orph = []
    off = 0.0
    for t, tk in enumerate(ticks):
        if t % 3 != 2:  # drop the re-registrations: nobody dies this tick
            keep = tk["ev_kind"] != synth.EV_REGISTER
            tk = dict(tk, **{k: tk[k][keep] for k in ("ev_kind", "ev_slot", "ev_val", "ev_ts", "ev_seq")})
        else:
            off += 0.4
        n = carried + tk["n_new"]
        args = (tk["now"] + off, 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"] + off, tk["ev_seq"], n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp(g, o, a, b, t)
        n_orph.append(len(b["orphans"]))
        carried = n + len(b["orphans"]) - len(b["assign"])
    wt, fb = g.window_stats()
    assert wt >= 6, "window ticks: %d (fallbacks %d)" % (wt, fb)
    assert all(n_orph[t] == 0 for t in range(len(ticks)) if t % 3 != 2)
    assert any(n_orph[t] > 0 for t in range(len(ticks)) if t % 3 == 2), n_orph
    g.close()


@pytest.mark.parametrize("seed", range(24))
def test_window_random_vs_oracle(seed, eager=False):
    """Every message kind and edge case of the random scenarios (register 0 / -1 of a
    queued worker, reconnects, unknown ids, repeated results, deaths between a slot's
    own messages) with window mode on; task counts vary so ticks alternate between
    window ticks, fallbacks (a fill level above 0, unserved fronts) and general ticks
    that read a window holding tombstones."""
    W = [300, 1000, 3000][seed % 3]
    scen = synth.random_scenario(9000 + seed, W=W, n_ticks=10, max_events=[50, 400, 1500][(seed // 3) % 3],
                                 max_new=[40, 150, 600, 4000][(seed // 9) % 3 + (seed % 2)])
    st = dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
              queue=scen["init_queue"], log=scen["init_log"])
    g, o = _pair(st, 2 * len(scen["init_log"]) + 60000, max_events=4096, eager=eager)
    carried = 0
    for t, tk in enumerate(scen["ticks"]):
        log = o.export()["log"]
        seq = np.full(len(tk["ev_kind"]), -1, np.int64)
        for i in np.nonzero(tk["ev_kind"] == synth.EV_RESULT)[0]:
            mine = np.nonzero(log == tk["ev_slot"][i])[0]
            if len(mine) and tk["ev_pick"][i] % 5 != 4:
                seq[i] = mine[tk["ev_pick"][i] % len(mine)]
        n = carried + tk["n_new"]
        args = (tk["now"], scen["tte"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp(g, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    g.close()


def test_window_relaunch_without_commit_is_identical():
    """A window tick reads only committed state: relaunched uncommitted it computes the
    same assignments, orphans and evicted slots; committed once, the state matches."""
    st, ticks = _stream(5, 8192, 1024, 0.3, n_ticks=3)
    E = max(len(t["ev_kind"]) for t in ticks)
    g, o = _pair(st, 2 * len(st["log"]) + 8 * 1024 + 16, max_events=E, purge_mode=2)
    carried = 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        outs = [g.tick(*args, commit=False) for _ in range(2)]
        for k in ("assign", "orphans", "evicted", "reconnect"):
            np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg="tick %d %s" % (t, k))
        g.commit()
        b = o.tick(*args)
        _cmp(g, o, outs[1], b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    assert g.window_stats()[0] >= 2


def test_window_device_view_is_dense():
    """The device view of a window context is the dense LRU queue (the window is
    rewritten from position 0 first), and ticks continue from it."""
    st, ticks = _stream(6, 4096, 256, 0.3, n_ticks=5)
    E = max(len(t["ev_kind"]) for t in ticks)
    g, o = _pair(st, 2 * len(st["log"]) + 8 * 256 + 16, max_events=E, purge_mode=2)
    carried = 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp(g, o, a, b, t)
        v = g.device_view()
        assert v.queue_len == len(o.export()["queue"])
        carried = n + len(b["orphans"]) - len(b["assign"])
    assert g.window_stats()[0] >= 2


def test_window_off_and_auto_agree():
    """The same stream with window ticks off, forced on and in auto mode (contexts of
    <= 128K workers: off): identical outputs."""
    st, ticks = _stream(7, 8192, 512, 0.3, n_ticks=5)
    E = max(len(t["ev_kind"]) for t in ticks)
    res = []
    for mode in (0, 1, -1):
        g = GpuBalancer(8192, 2 * len(st["log"]) + 6 * 512 + 16, max_events=E)
        g.set_window(mode)
        g.load(st)
        carried, outs = 0, []
        for tk in ticks:
            n = carried + tk["n_new"]
            a = g.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
            outs.append(a)
            carried = n + len(a["orphans"]) - len(a["assign"])
        res.append((outs, g.read_state(), g.window_stats()))
        g.close()
    assert res[0][2][0] == 0 and res[1][2][0] >= 3 and res[2][2][0] == 0
    for outs, sg, _ in res[1:]:
        for a, b in zip(res[0][0], outs):
            for k in ("assign", "orphans", "evicted", "reconnect"):
                np.testing.assert_array_equal(a[k], b[k])
        for k in ("queue", "reg", "log"):
            np.testing.assert_array_equal(res[0][1][k], sg[k])


@pytest.mark.parametrize("seed,W,T,dt", [(8, 8192, 512, 0.3), (9, 20000, 2048, 0.05)])
def test_window_stream_deferred_commits(seed, W, T, dt):
    """Ticks back to back with no state read in between, so every commit is deferred
    into the next tick's first launch (the window commit's tomb list and its count must
    survive that launch's clears); outputs compared every tick, the state at the end."""
    st, ticks = _stream(seed, W, T, dt, n_ticks=10)
    E = max(len(t["ev_kind"]) for t in ticks)
    g, o = _pair(st, 3 * len(st["log"]) + 20 * T + 16, max_events=E, purge_mode=2)
    carried = 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        a, b = g.tick(*args), o.tick(*args)
        for k in ("reconnect", "assign", "orphans", "evicted"):
            np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))
        carried = n + len(b["orphans"]) - len(b["assign"])
    _cmp(g, o, a, b, len(ticks) - 1)
    assert g.window_stats()[0] >= 5
    g.close()


@pytest.mark.parametrize("seed", range(0, 24, 3))
def test_window_random_eager_vs_oracle(seed):
    """The random scenarios with eager commits: fallbacks, reruns through the sort and
    general ticks must leave the eagerly enqueued commit without effect."""
    test_window_random_vs_oracle(seed, eager=True)


def test_eager_tick_cannot_be_relaunched_uncommitted():
    """An eagerly committed tick must be waited for and committed before the next launch
    (a tick committed the ordinary way may still be relaunched uncommitted)."""
    st, ticks = _stream(10, 8192, 512, 0.3, n_ticks=4)
    E = max(len(t["ev_kind"]) for t in ticks)
    g, o = _pair(st, 2 * len(st["log"]) + 8 * 512 + 16, max_events=E, purge_mode=2, eager=True)
    carried, raised = 0, 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        a = g.tick(*args, commit=False)
        try:
            g.launch(*args)
        except FaasbalError as e:
            assert "eagerly" in str(e)
            raised += 1
        else:
            a2 = g.wait()
            assert a2["n_assigned"] == a["result"]["n_assigned"]
        g.commit()
        b = o.tick(*args)
        _cmp(g, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    assert raised >= 2
    g.close()


@pytest.mark.parametrize("eager", [False, True], ids=["deferred", "eager"])
def test_window_state_reads_refused_until_commit(eager):
    """fb_read_state / fb_device_view_get / fb_read_inflight between the launch and the
    commit of a window tick fail with FB_ESTATE (the window moves at the commit, on the
    device already with eager commits); after the commit they read the new state and the
    stream continues identical to the oracle."""
    st, ticks = _stream(5, 4096, 256, 0.3, n_ticks=4)
    E = max(len(t["ev_kind"]) for t in ticks)
    g, o = _pair(st, 2 * len(st["log"]) + 8 * 256 + 16, max_events=E, purge_mode=2)
    g.set_eager_commit(eager)
    carried, refused = 0, 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        g.launch(*args)
        res = g.wait()
        a = dict(result=res, reconnect=g.event_status(), assign=g.assignments(), orphans=g.orphans(),
                 evicted=g.evicted())
        win, r_t = g.window_stats()[0], 0
        for read in (g.read_state, g.device_view, g.inflight):
            try:
                read()
            except FaasbalError as e:
                assert e.code == _lib.FB_ESTATE
                r_t += 1
        g.commit()
        b = o.tick(*args)
        _cmp(g, o, a, b, t)
        assert r_t == (3 if g.window_stats()[0] > win else 0), (t, r_t)
        refused += r_t
        carried = n + len(b["orphans"]) - len(b["assign"])
    assert refused >= 3
    g.close()


def _large_stream(g, o, ticks, eager):
    g.set_eager_commit(eager)
    carried, n_orph = 0, 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        a, b = g.tick(*args), o.tick(*args)
        for k in ("reconnect", "assign", "orphans", "evicted"):
            np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))
        n_orph += len(b["orphans"])
        carried = n + len(b["orphans"]) - len(b["assign"])
    sg, so = g.read_state(), o.export()
    for k in ("reg", "queue", "log"):
        np.testing.assert_array_equal(sg[k], so[k], err_msg=k)
    m = so["reg"].astype(bool)
    np.testing.assert_array_equal(sg["free"][m], so["free"][m])
    np.testing.assert_array_equal(sg["hb"][m], so["hb"][m])
    return n_orph


@pytest.mark.parametrize("eager", [False, True], ids=["deferred", "eager"])
def test_large_table_window_stream_vs_oracle(eager):
    """Large tables (> 128K workers, auto mode, no in-flight counts: results clear their
    log entries in place): window ticks whose k_logscan tests the log against the died
    bitmap through its one-bit-per-word summary.  Every output and the state equal the
    oracle's; deaths happen inside window ticks."""
    W = 160_000
    st = synth.zipf_state(W=W, seed=8, dead_frac=0.0)
    ticks = synth.stream_ticks(st, n_ticks=6, seed=9, tasks_per_tick=8192, results_per_tick=8192, dt=0.15)
    E = max(len(t["ev_kind"]) for t in ticks)
    cap = len(st["log"]) + 16 * 8192
    g = GpuBalancer(W, cap, max_events=E)
    g.load(st)
    o = Oracle(W, cap, purge_mode=2)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    n_orph = _large_stream(g, o, ticks, eager)
    wt, fb = g.window_stats()
    assert wt >= 3 and n_orph > 0, (wt, fb, n_orph)
    g.close()


@pytest.mark.parametrize("seed", range(0, 24, 4))
def test_window_random_ticketed_chunks_vs_oracle(monkeypatch, seed):
    """k_emit_win with its chunks taken by ticket (fb_set_path("win_direct", 0): the form
    for grids too large to be resident at once) instead of by workgroup index."""
    from faasbal.balancer import TEST_PATHS
    monkeypatch.setitem(TEST_PATHS, "win_direct", 0)
    test_window_random_vs_oracle(seed)


@pytest.mark.parametrize("seed", range(1, 24, 6))
def test_window_random_four_slot_tiles_vs_oracle(monkeypatch, seed):
    """The slot purge in k_ev_apply_ll (and k_scan) with four 256-slot tiles per workgroup
    (fb_set_path("wtiles", 4), the default from 1024 tiles) on small tables."""
    from faasbal.balancer import TEST_PATHS
    monkeypatch.setitem(TEST_PATHS, "wtiles", 4)
    test_window_random_vs_oracle(seed)


def test_window_stream_four_slot_tiles_vs_oracle(monkeypatch):
    """configs[4]'s event mix (20 000 slots: 79 tiles, a partial last group of four) with
    the four-tile slot purge forced."""
    from faasbal.balancer import TEST_PATHS
    monkeypatch.setitem(TEST_PATHS, "wtiles", 4)
    test_window_stream_vs_oracle(3, 20000, 2048, 0.05, False)
