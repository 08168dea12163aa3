"""The C oracle (oracle/push_oracle.c) against golden vectors captured from the
unmodified reference loop (tests/golden/make_golden.py).  CPU only."""
import glob
import os

import numpy as np
import pytest

from oracle import DequeOracle, Oracle, fixture_expect, fixture_ticks

GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if not os.path.basename(p).startswith("deque_"))  # start_heartbeat vectors


def replay(z, purge_mode):
    W = int(z["W"])
    total_new = int(len(z["exp_assign"]))
    o = Oracle(W, len(z["init_log"]) + total_new + 16, purge_mode=purge_mode)
    o.load(z["init_reg"], z["init_free"], z["init_hb"], z["init_epoch"], z["init_queue"], z["init_log"])
    carried = 0
    for t, tk in enumerate(fixture_ticks(z)):
        exp = fixture_expect(z, t)
        n_pending = carried + tk["n_new"]
        out = o.tick(tk["now"], float(z["tte"]), tk["ev_kind"], tk["ev_slot"], tk["ev_val"],
                     tk["ev_ts"], tk["ev_seq"], n_pending)
        st = o.export()
        yield t, exp, out, st, n_pending
        carried = n_pending + len(out["orphans"]) - len(out["assign"])


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
@pytest.mark.parametrize("purge_mode", [0, 1, 2])
def test_oracle_matches_reference(path, purge_mode):
    z = np.load(path)
    if purge_mode == 0 and int(z["W"]) > 1024:
        pytest.skip("as-written purge is O(W) per iteration; covered by purge_mode=1")
    for t, exp, out, st, n_pending in replay(z, purge_mode):
        assert n_pending + len(out["orphans"]) == exp["n_pending"], t
        np.testing.assert_array_equal(out["reconnect"], exp["reconnect"], err_msg=f"tick {t}")
        np.testing.assert_array_equal(out["orphans"], exp["orphans"], err_msg=f"tick {t}")
        np.testing.assert_array_equal(out["assign"], exp["assign"], err_msg=f"tick {t}")
        np.testing.assert_array_equal(out["evicted"], exp["evicted"], err_msg=f"tick {t}")
        np.testing.assert_array_equal(st["reg"], exp["post_reg"], err_msg=f"tick {t}")
        reg = exp["post_reg"].astype(bool)
        np.testing.assert_array_equal(st["free"][reg], exp["post_free"][reg], err_msg=f"tick {t}")
        np.testing.assert_array_equal(st["hb"][reg], exp["post_hb"][reg], err_msg=f"tick {t}")
        np.testing.assert_array_equal(st["queue"], exp["post_queue"], err_msg=f"tick {t}")


DEQUE = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "deque_*.npz")))


@pytest.mark.parametrize("path", DEQUE, ids=[os.path.basename(p)[:-4] for p in DEQUE])
def test_deque_oracle_matches_reference(path):
    """deque_oracle.c against vectors captured from the reference's start() loop
    (task_dispatcher.py:251-322): duplicate deque entries, no heartbeats."""
    z = np.load(path)
    W = int(z["W"])
    o = DequeOracle(W, len(z["init_log"]) + len(z["exp_assign"]) + 16)
    o.load(z["init_reg"], z["init_free"], z["init_hb"], z["init_epoch"], z["init_queue"], z["init_log"])
    carried = 0
    for t, tk in enumerate(fixture_ticks(z)):
        exp = fixture_expect(z, t)
        n_pending = carried + tk["n_new"]
        out = o.tick(tk["now"], float(z["tte"]), tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"],
                     tk["ev_seq"], n_pending)
        st = o.export()
        assert n_pending == exp["n_pending"], t
        assert not exp["reconnect"].any() and not len(exp["orphans"]) and not len(exp["evicted"])
        np.testing.assert_array_equal(out["reconnect"], exp["reconnect"], err_msg=f"tick {t}")
        np.testing.assert_array_equal(out["assign"], exp["assign"], err_msg=f"tick {t}")
        np.testing.assert_array_equal(st["reg"], exp["post_reg"], err_msg=f"tick {t}")
        reg = exp["post_reg"].astype(bool)
        np.testing.assert_array_equal(st["free"][reg], exp["post_free"][reg], err_msg=f"tick {t}")
        np.testing.assert_array_equal(st["hb"][reg], exp["post_hb"][reg], err_msg=f"tick {t}")
        np.testing.assert_array_equal(st["queue"], exp["post_queue"], err_msg=f"tick {t}")
        carried = n_pending - len(out["assign"])


def test_deque_fixtures_hold_duplicates():
    """The start() vectors exercise the deque's repeated ids (the case the GPU
    handles with per-token ranks)."""
    n = 0
    for path in DEQUE:
        z = np.load(path)
        q = z["exp_post_queue"]
        off = z["exp_post_queue_off"]
        for t in range(int(z["n_ticks"])):
            seg = q[off[t]:off[t + 1]]
            n += len(seg) - len(np.unique(seg))
    assert n > 20


@pytest.mark.parametrize("seed", range(12))
def test_heap_purge_equals_scan(seed):
    """purge_mode 2 (min-heap of heartbeats) deletes exactly the records the O(W)
    scan of purge_workers (task_dispatcher.py:241-249) deletes: random streams with
    per-event clocks, every output and the exported state compared."""
    from faasbal import synth
    scen = synth.random_scenario(100 + seed, W=64, n_ticks=6, max_events=120, max_new=150)
    outs = []
    for mode in (1, 2):
        o = Oracle(scen["W"], len(scen["init_log"]) + 4096, purge_mode=mode)
        o.load(scen["init_reg"], scen["init_free"], scen["init_hb"], scen["init_epoch"], scen["init_queue"],
               scen["init_log"])
        res, carried = [], 0
        for tk in scen["ticks"]:
            n = carried + tk["n_new"]
            r = o.tick(tk["now"], scen["tte"], tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"],
                       tk["ev_seq"], n)
            res.append(r)
            carried = n + len(r["orphans"]) - len(r["assign"])
        outs.append((res, o.export()))
    (ra, sa), (rb, sb) = outs
    for a, b in zip(ra, rb):
        for k in ("reconnect", "assign", "orphans", "evicted"):
            np.testing.assert_array_equal(a[k], b[k])
    for k in ("reg", "free", "queue", "log"):
        np.testing.assert_array_equal(sa[k], sb[k])
