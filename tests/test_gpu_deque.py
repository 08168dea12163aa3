"""Deque contexts (the loop without heartbeats, PushDispatcher.start,
reference task_dispatcher.py:251-322) through the C ABI vs the deque oracle and
the golden vectors captured from the reference start() loop.

Bit-exact on every output: per-event status, task -> slot assignments and the
post-tick state (registered, free_processes, the deque with its repeated ids,
in-flight log).
"""
import glob
import os

import numpy as np
import pytest

from faasbal import FaasbalError, GpuBalancer, synth
from faasbal.balancer import TEST_PATHS
from oracle import DequeOracle, fixture_expect, fixture_ticks

pytestmark = pytest.mark.gpu
DEQUE = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "deque_*.npz")))


def _pair(st, log_cap, max_events=4096, max_tokens=None):
    W = len(st["reg"])
    g = GpuBalancer(W, log_cap, max_events=max_events, mode="deque", max_tokens=max_tokens)
    g.load(st)
    o = DequeOracle(W, log_cap)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    return g, o


def _cmp(g, o, a, b, t):
    for k in ("reconnect", "assign"):
        np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))
    assert len(a["orphans"]) == 0 and len(a["evicted"]) == 0
    sg, so = g.read_state(), o.export()
    np.testing.assert_array_equal(sg["reg"], so["reg"], err_msg="tick %d reg" % t)
    reg = so["reg"].astype(bool)
    np.testing.assert_array_equal(sg["free"][reg], so["free"][reg], err_msg="tick %d free" % t)
    np.testing.assert_array_equal(sg["hb"][reg], so["hb"][reg], err_msg="tick %d hb" % t)
    np.testing.assert_array_equal(sg["queue"], so["queue"], err_msg="tick %d queue" % t)
    np.testing.assert_array_equal(sg["log"], so["log"], err_msg="tick %d log" % t)


@pytest.mark.parametrize("path", DEQUE, ids=[os.path.basename(p)[:-4] for p in DEQUE])
def test_deque_golden_replay(path):
    z = np.load(path)
    W = int(z["W"])
    cap = len(z["init_log"]) + len(z["exp_assign"]) + 16
    g = GpuBalancer(W, cap, max_events=max(1, int(np.diff(z["ev_off"]).max(initial=0))), mode="deque")
    g.load_state(z["init_reg"], z["init_free"], z["init_hb"], z["init_epoch"], z["init_queue"], z["init_log"])
    carried = 0
    for t, tk in enumerate(fixture_ticks(z)):
        exp = fixture_expect(z, t)
        n = carried + tk["n_new"]
        out = g.tick(tk["now"], 0.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        np.testing.assert_array_equal(out["reconnect"], exp["reconnect"], err_msg="tick %d status" % t)
        np.testing.assert_array_equal(out["assign"], exp["assign"], err_msg="tick %d assign" % t)
        st = g.read_state(with_log=False)
        np.testing.assert_array_equal(st["queue"], exp["post_queue"], err_msg="tick %d queue" % t)
        np.testing.assert_array_equal(st["reg"], exp["post_reg"], err_msg="tick %d reg" % t)
        reg = exp["post_reg"].astype(bool)
        np.testing.assert_array_equal(st["free"][reg], exp["post_free"][reg])
        np.testing.assert_array_equal(st["hb"][reg], exp["post_hb"][reg])
        carried = n - len(out["assign"])


def _resolve_seq(log, tk):
    seq = np.full(len(tk["ev_kind"]), -1, np.int64)
    for i in np.nonzero(tk["ev_kind"] == synth.EV_RESULT)[0]:
        mine = np.nonzero(log == tk["ev_slot"][i])[0]
        if len(mine) and tk["ev_pick"][i] % 5 != 4:
            seq[i] = mine[tk["ev_pick"][i] % len(mine)]
    return seq


@pytest.mark.parametrize("seed", range(30))
def test_deque_random_multitick_vs_oracle(seed):
    """Repeated ids in the deque (up to 3x the distinct ones), registers with
    0/-1, results bringing a worker back to 1 free process, ignored kinds."""
    scen = synth.random_deque_scenario(700 + seed, W=[5, 37, 300, 1000][seed % 4], n_ticks=6,
                                       max_events=[20, 200, 2000][seed % 3], max_new=[50, 400, 3000][(seed // 3) % 3],
                                       dup_frac=[0.3, 1.0, 3.0][(seed // 9) % 3])
    st = dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
              queue=scen["init_queue"], log=scen["init_log"])
    g, o = _pair(st, len(st["log"]) + 40000, max_tokens=8 * scen["W"] + 4096)
    carried = 0
    for t, tk in enumerate(scen["ticks"]):
        seq = _resolve_seq(o.export()["log"], tk)
        n = carried + tk["n_new"]
        args = (tk["now"], 0.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        a, b = g.tick(*args), o.tick(*args)
        _cmp(g, o, a, b, t)
        carried = n - len(b["assign"])


def test_deque_config3_with_duplicates():
    """configs[2] loads (1M tasks x 64K workers) without heartbeats; 2 % of the
    queued workers hold a second deque entry."""
    st = synth.zipf_deque_state(W=65536, seed=0, dup_frac=0.02)
    T = 1_000_000
    g, o = _pair(st, len(st["log"]) + T + 16, max_events=1)
    a = g.tick(1000.0, 0.0, n_pending=T)
    b = o.tick(1000.0, 0.0, [], [], [], [], [], T)
    assert a["result"]["n_assigned"] == T
    _cmp(g, o, a, b, 0)


def test_deque_unknown_result_is_reported():
    st = dict(reg=np.array([1, 0, 1], np.uint8), free=np.array([2, 0, 0], np.int32), hb=np.zeros(3),
              epoch=np.zeros(3, np.uint32), queue=np.array([0], np.int32), log=np.zeros(0, np.int32))
    g, o = _pair(st, 1000)
    args = (1.0, 0.0, [synth.EV_RESULT, synth.EV_RESULT, synth.EV_HEARTBEAT], [1, 2, 1], [0, 0, 0],
            [0.5, 0.6, 0.7], [-1, -1, -1], 10)
    a, b = g.tick(*args), o.tick(*args)
    np.testing.assert_array_equal(a["reconnect"], [2, 0, 0])
    _cmp(g, o, a, b, 0)


def test_deque_capacity_is_an_error():
    W = 4
    st = dict(reg=np.ones(W, np.uint8), free=np.full(W, 5, np.int32), hb=np.zeros(W), epoch=np.zeros(W, np.uint32),
              queue=np.arange(W, dtype=np.int32), log=np.zeros(0, np.int32))
    g = GpuBalancer(W, 1000, max_events=64, mode="deque", max_tokens=6)
    g.load(st)
    with pytest.raises(FaasbalError):
        g.tick(1.0, 0.0, [synth.EV_REGISTER] * 4, [0, 1, 2, 3], [5] * 4, [0.1, 0.2, 0.3, 0.4], [-1] * 4, 0)


def test_deque_relaunch_without_commit_is_identical():
    st = synth.zipf_deque_state(W=4096, seed=5, dup_frac=0.1)
    g = GpuBalancer(4096, len(st["log"]) + 200_000, mode="deque")
    g.load(st)
    outs = []
    for _ in range(3):
        g.launch(1000.0, 0.0, n_pending=50_000)
        g.wait()
        outs.append(g.assignments())
    for x in outs[1:]:
        np.testing.assert_array_equal(outs[0], x)


@pytest.fixture
def force_plan(monkeypatch):
    monkeypatch.setitem(TEST_PATHS, "plan", 1)


@pytest.mark.parametrize("seed", range(6))
def test_deque_random_plan_path(force_plan, seed):
    test_deque_random_multitick_vs_oracle(seed + 10)


def test_deque_config3_plan_path(force_plan):
    test_deque_config3_with_duplicates()


@pytest.mark.parametrize("seed", range(3))
def test_deque_random_chunked_emit(monkeypatch, seed):
    monkeypatch.setitem(TEST_PATHS, "plan", 2)
    test_deque_random_multitick_vs_oracle(seed + 20)
