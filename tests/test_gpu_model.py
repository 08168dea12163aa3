"""The GPU tick *algorithm* (numpy model in tests/gpu_model.py) against the
golden vectors and the sequential oracle.  CPU only: validates the
decomposition the kernels implement, independent of HIP."""
import glob
import os

import numpy as np
import pytest

import gpu_model
from oracle import fixture_expect, fixture_ticks

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "small_*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_model_matches_reference(path):
    z = np.load(path)
    st = dict(reg=z["init_reg"], free=z["init_free"], hb=z["init_hb"], epoch=z["init_epoch"],
              queue=z["init_queue"], log=z["init_log"])
    carried = 0
    for t, tk in enumerate(fixture_ticks(z)):
        exp = fixture_expect(z, t)
        n_pending = carried + tk["n_new"]
        out, st = gpu_model.tick(st, tk["now"], float(z["tte"]), tk["ev_kind"], tk["ev_slot"], tk["ev_val"],
                                 tk["ev_ts"], tk["ev_seq"], n_pending)
        for k in ("reconnect", "assign", "orphans", "evicted"):
            np.testing.assert_array_equal(out[k], exp[k], err_msg="tick %d %s" % (t, k))
        np.testing.assert_array_equal(st["queue"], exp["post_queue"])
        np.testing.assert_array_equal(st["reg"], exp["post_reg"])
        reg = exp["post_reg"].astype(bool)
        np.testing.assert_array_equal(st["free"][reg], exp["post_free"][reg])
        np.testing.assert_array_equal(st["hb"][reg], exp["post_hb"][reg])
        carried = n_pending + len(out["orphans"]) - len(out["assign"])


DEQUE = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "deque_*.npz")))


def _deque_run(st, ticks, o):
    st = gpu_model.deque_load(st)
    carried = 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        seq = tk.get("ev_seq", np.full(len(tk["ev_kind"]), -1, np.int64))
        out, st = gpu_model.tick_deque(st, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        exp = o.tick(0.0, 0.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, n)
        for k in ("reconnect", "assign"):
            np.testing.assert_array_equal(out[k], exp[k], err_msg="tick %d %s" % (t, k))
        so = o.export()
        np.testing.assert_array_equal(st["queue"], so["queue"], err_msg="tick %d queue" % t)
        reg = so["reg"].astype(bool)
        np.testing.assert_array_equal(st["free"][reg], so["free"][reg], err_msg="tick %d free" % t)
        np.testing.assert_array_equal(st["log"], so["log"], err_msg="tick %d log" % t)
        carried = n - len(out["assign"])


@pytest.mark.parametrize("seed", range(60))
def test_deque_model_matches_oracle(seed):
    """Token ranks (per-slot counts, part-1/part-2 fix-ups) reproduce the
    sequential start() loop on random streams with repeated deque ids."""
    from faasbal import synth
    from oracle import DequeOracle
    scen = synth.random_deque_scenario(500 + seed, W=[5, 12, 30][seed % 3], n_ticks=6,
                                       max_events=[10, 40, 120][(seed // 3) % 3], max_new=[20, 80, 400][seed % 3],
                                       dup_frac=[0.3, 1.0, 3.0][(seed // 9) % 3])
    st = dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
              queue=scen["init_queue"], log=scen["init_log"])
    o = DequeOracle(scen["W"], len(st["log"]) + 10000)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    _deque_run(st, scen["ticks"], o)


@pytest.mark.parametrize("path", DEQUE, ids=[os.path.basename(p)[:-4] for p in DEQUE])
def test_deque_model_matches_reference(path):
    from oracle import DequeOracle
    z = np.load(path)
    st = dict(reg=z["init_reg"], free=z["init_free"], hb=z["init_hb"], epoch=z["init_epoch"],
              queue=z["init_queue"], log=z["init_log"])
    o = DequeOracle(int(z["W"]), len(z["init_log"]) + len(z["exp_assign"]) + 16)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    _deque_run(st, list(fixture_ticks(z)), o)
