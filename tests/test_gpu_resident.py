"""Device-resident message batches (fb_tick_stage of arrays in the GPU's memory) vs the
oracle (task_dispatcher.py:324-419 restated).

A batch already in HBM -- parsed there, or copied ahead as bench.py's stream workload
does -- is read in place by the tick and checked by its first kernel (k_ev_link): the
outputs and the post-tick state must equal the oracle's on every tick, window ticks
included; an invalid message fails the tick at wait naming its index (the first one),
nothing is committed and the next tick runs.
"""
import numpy as np
import pytest

from faasbal import GpuBalancer, FaasbalError, synth
from oracle import Oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _dev(*arrs):
    return [None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0") for a in arrs]


def _tick_dev(g, now, tte, k, s, v, t, q, n):
    d = _dev(k, s, v, t, q)  # held until the tick was waited for
    g.stage_device(now, *d)
    g.launch_staged(tte, n)
    r = g.wait()
    del d
    out = dict(result=r, reconnect=g.event_status(), assign=g.assignments(), orphans=g.orphans(),
               evicted=g.evicted())
    g.commit()
    return out


def _cmp(g, o, a, b, t):
    for k in ("reconnect", "assign", "orphans", "evicted"):
        np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))
    sg, so = g.read_state(), o.export()
    for k in ("reg", "queue", "log"):
        np.testing.assert_array_equal(sg[k], so[k], err_msg="tick %d %s" % (t, k))
    reg = so["reg"].astype(bool)
    np.testing.assert_array_equal(sg["free"][reg], so["free"][reg], err_msg="tick %d free" % t)
    np.testing.assert_array_equal(sg["hb"][reg], so["hb"][reg], err_msg="tick %d hb" % t)


@pytest.mark.parametrize("window", [1, 0])
def test_resident_stream_vs_oracle(window):
    """configs[4]'s event mix at reduced size from HBM-resident batches, with window
    ticks forced on and off."""
    W, T = 8192, 512
    st = synth.zipf_state(W=W, seed=11, dead_frac=0.0)
    ticks = synth.stream_ticks(st, n_ticks=8, seed=18, tasks_per_tick=T, results_per_tick=T, dt=0.5,
                               hb_frac=0.01, join_frac=0.002)
    E = max(len(t["ev_kind"]) for t in ticks)
    g = GpuBalancer(W, 3 * len(st["log"]) + 20 * T + 16, max_events=E)
    g.set_window(window)
    g.load(st)
    o = Oracle(W, 3 * len(st["log"]) + 20 * T + 16, purge_mode=2)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    carried = 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        a = _tick_dev(g, tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        b = o.tick(tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        _cmp(g, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    if window:
        assert g.window_stats()[0] >= 4
    g.close()


def test_resident_random_scenario_without_seq():
    """Every message kind of the random scenarios (reconnects, unknown ids, register 0 /
    -1), seq omitted on ticks without results (filled with -1 on the device)."""
    scen = synth.random_scenario(4242, W=1000, n_ticks=8, max_events=400, max_new=300)
    st = dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
              queue=scen["init_queue"], log=scen["init_log"])
    g = GpuBalancer(1000, 2 * len(scen["init_log"]) + 60000, max_events=4096)
    g.load(st)
    o = Oracle(1000, 2 * len(scen["init_log"]) + 60000)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    carried = 0
    for t, tk in enumerate(scen["ticks"]):
        keep = tk["ev_kind"] != synth.EV_RESULT  # no results: seq may be omitted
        k, s, v, ts = tk["ev_kind"][keep], tk["ev_slot"][keep], tk["ev_val"][keep], tk["ev_ts"][keep]
        n = carried + tk["n_new"]
        a = _tick_dev(g, tk["now"], scen["tte"], k, s, v, ts, None, n)
        b = o.tick(tk["now"], scen["tte"], k, s, v, ts, np.full(len(k), -1, np.int64), n)
        _cmp(g, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    g.close()


@pytest.mark.parametrize("bad", ["decreasing", "future", "slot", "kind", "two"])
def test_invalid_messages_in_resident_batches(bad):
    """An invalid message of a device batch fails the tick at wait naming the first
    offending index; nothing is committed and the next tick matches the oracle."""
    st = synth.uniform_state(W=64, seed=1)
    g = GpuBalancer(64, 4000, max_events=4096)
    g.load(st)
    o = Oracle(64, 4000)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    ts = np.array([999.0, 999.5, 998.0 if bad == "decreasing" else 999.6, 999.7])
    kinds = np.array([2, 2, 2, 2], np.uint8)
    slots = np.array([1, 2, 3, 4], np.int32)
    if bad == "future":
        ts[3] = 1000.5
    if bad in ("slot", "two"):
        slots[2] = 1 << 20
    if bad in ("kind", "two"):
        kinds[3] = 9
    first = 2 if bad in ("decreasing", "slot", "two") else 3
    with pytest.raises(FaasbalError, match="event %d" % first):
        _tick_dev(g, 1000.0, 10.0, kinds, slots, np.zeros(4, np.int32), ts, np.full(4, -1, np.int64), 10)
    args = (1000.0, 10.0, np.array([2], np.uint8), np.array([5], np.int32), np.zeros(1, np.int32),
            np.array([999.0]), np.full(1, -1, np.int64), 10)
    a, b = _tick_dev(g, *args), o.tick(*args)
    _cmp(g, o, a, b, 0)
    g.close()


def test_mixed_memory_batch_rejected():
    """Arrays partly in GPU memory, partly on the host: refused at stage."""
    g = GpuBalancer(64, 4000, max_events=64)
    g.load(synth.uniform_state(W=64, seed=1))
    k, s, v, t, q = _dev(np.array([2], np.uint8), np.array([1], np.int32), np.zeros(1, np.int32),
                         np.array([999.0]), np.full(1, -1, np.int64))
    ht = np.array([999.0])
    with pytest.raises(FaasbalError, match="mix"):
        g._chk(g.lib.fb_tick_stage(g.h, 1000.0, 1, k.data_ptr(), s.data_ptr(), v.data_ptr(), ht.ctypes.data,
                                   q.data_ptr()))
    g.close()
