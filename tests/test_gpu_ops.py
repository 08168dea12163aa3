"""The per-operation C ABI forms (fb_apply_events, fb_purge, fb_assign), called
through ctypes, against the oracle driven the same way: messages with nothing
dispatched (dispatch_limit 0) and the purge at the last message's clock; a purge
at `now`; a dispatch of n tasks with its purge.  Bit-exact on every output and on
the committed state."""
import ctypes as C

import numpy as np
import pytest

from faasbal import GpuBalancer, synth
from faasbal._lib import TickResult
from oracle import Oracle

pytestmark = pytest.mark.gpu


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _pair(st, cap, E):
    W = len(st["reg"])
    g = GpuBalancer(W, cap, max_events=E)
    g.load(st)
    o = Oracle(W, cap)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    return g, o


def _state_eq(g, o):
    sg, so = g.read_state(), o.export()
    reg = so["reg"].astype(bool)
    np.testing.assert_array_equal(sg["reg"], so["reg"])
    np.testing.assert_array_equal(sg["free"][reg], so["free"][reg])
    np.testing.assert_array_equal(sg["hb"][reg], so["hb"][reg])
    np.testing.assert_array_equal(sg["queue"], so["queue"])
    np.testing.assert_array_equal(sg["log"], so["log"])


@pytest.mark.parametrize("seed", range(6))
def test_apply_purge_assign_vs_oracle(seed):
    scen = synth.random_scenario(900 + seed, W=300, n_ticks=4, max_events=300, max_new=500)
    st = dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
              queue=scen["init_queue"], log=scen["init_log"])
    tte = float(scen["tte"])
    g, o = _pair(st, len(st["log"]) + 8 * 1200 + 64, 512)
    lib, h = g.lib, g.h
    for tk in scen["ticks"]:
        kind = np.ascontiguousarray(tk["ev_kind"], np.uint8)
        slot = np.ascontiguousarray(tk["ev_slot"], np.int32)
        val = np.ascontiguousarray(tk["ev_val"], np.int32)
        ts = np.ascontiguousarray(tk["ev_ts"], np.float64)
        seq = np.ascontiguousarray(tk["ev_seq"], np.int64)
        E = len(kind)
        # 1) the messages alone: purge after the last one at its clock, nothing dispatched
        r = TickResult()
        evs = np.zeros(max(E, 1), np.uint8)
        orph = np.zeros(4096, np.int64)
        evic = np.zeros(512, np.int32)
        assert lib.fb_apply_events(h, tte, E, _p(kind), _p(slot), _p(val), _p(ts), _p(seq), C.byref(r), _p(evs),
                                   _p(orph), _p(evic)) == 0, g.lib.fb_last_error(h)
        if E:
            x = o.tick(float(ts[-1]), tte, kind, slot, val, ts, seq, 0, dispatch_limit=0)
            np.testing.assert_array_equal(evs[:E], x["reconnect"])
            np.testing.assert_array_equal(orph[:r.n_orphans], x["orphans"])
            np.testing.assert_array_equal(evic[:r.n_evicted], x["evicted"])
            assert r.n_assigned == 0
        _state_eq(g, o)
        now = float(tk["now"])
        # 2) purge_workers at now
        r = TickResult()
        assert lib.fb_purge(h, now, tte, C.byref(r), _p(orph), _p(evic)) == 0
        x = o.tick(now, tte, [], [], [], [], np.zeros(0, np.int64), 0, dispatch_limit=0)
        np.testing.assert_array_equal(orph[:r.n_orphans], x["orphans"])
        np.testing.assert_array_equal(evic[:r.n_evicted], x["evicted"])
        _state_eq(g, o)
        # 3) the dispatch block for n tasks (the purge at now again: idempotent)
        n = int(tk["n_new"])
        r = TickResult()
        asg = np.zeros(max(n, 1) + 4096, np.int32)
        assert lib.fb_assign(h, now, tte, n, C.byref(r), _p(asg), _p(orph), _p(evic)) == 0
        x = o.tick(now, tte, [], [], [], [], np.zeros(0, np.int64), n)
        np.testing.assert_array_equal(asg[:r.n_assigned], x["assign"])
        _state_eq(g, o)
    g.close()
