"""BASELINE.json configs at their stated sizes.

* configs[2] (1M tasks x 64K workers, Zipf loads, 5 % dead): the oracle and the
  HIP tick against digests captured from the REFERENCE loop itself
  (``tests/golden/cfg2_full_digests.json``, ``make_golden.py cfg2full``: the
  unmodified ``task_dispatcher.py:324-419`` with a purge once per unchanged clock).
* configs[4] (64K new tasks per tick against 1M workers with churn): committed
  ticks, the HIP path against the oracle, bit-exact on every output.
* configs[3] (16M tasks x 1M workers): the oracle and the one-GPU HIP tick against
  digests captured from the reference loop the same way (``cfg3_full_digests.json``,
  ``make_golden.py cfg3full``); sharded over world 2 / 4 / 8: one tick of the rank
  contexts (single process, exchange summed on the device) against the oracle.
"""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(HERE, "golden"))

from faasbal import synth  # noqa: E402
from make_golden import digests  # noqa: E402  (pure numpy: no reference code is loaded)

CFG2 = json.load(open(os.path.join(HERE, "golden", "cfg2_full_digests.json")))
CFG3 = json.load(open(os.path.join(HERE, "golden", "cfg3_full_digests.json")))
CFG1 = json.load(open(os.path.join(HERE, "golden", "cfg1_full_digests.json")))


def _cfg2_state(fx=CFG2):
    p = fx["params"]
    gen = synth.uniform_state if p.get("loads") == "uniform" else synth.zipf_state
    return p, gen(W=p["W"], seed=p["seed"])


def _check(d, where, fx=CFG2):
    for k, v in fx["digests"].items():
        assert d[k] == v, "%s: %s differs from the reference capture (%s)" % (where, k, d[k])


def test_oracle_cfg2_full_matches_reference():
    from oracle import Oracle
    p, st = _cfg2_state()
    o = Oracle(p["W"], len(st["log"]) + p["T"] + len(st["log"]) + 16, purge_mode=1)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    out = o.tick(p["now"], p["tte"], [], [], [], [], [], p["T"])
    so = o.export()
    _check(digests(out["assign"], out["orphans"], out["evicted"], so["reg"], so["free"], so["hb"], so["queue"]),
           "oracle")


@pytest.mark.gpu
def test_gpu_cfg2_full_matches_reference():
    from faasbal import GpuBalancer
    p, st = _cfg2_state()
    g = GpuBalancer(p["W"], 2 * len(st["log"]) + p["T"] + 16, max_events=1, device=0)
    g.load(st)
    out = g.tick(p["now"], p["tte"], n_pending=p["T"])
    sg = g.read_state(with_log=False)
    assert out["result"]["n_assigned"] == CFG2["n_assigned"]
    _check(digests(out["assign"], out["orphans"], out["evicted"], sg["reg"], sg["free"], sg["hb"], sg["queue"]),
           "HIP tick")
    g.close()


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_oracle_full_matches_reference(name):
    """The oracle at configs[1]'s (100K tasks x 1K workers, uniform loads) and configs[3]'s
    (16M tasks x 1M workers) sizes, one tick, against the reference loop's own outputs."""
    fx = dict(cfg1=CFG1, cfg3=CFG3)[name]
    from oracle import Oracle
    p, st = _cfg2_state(fx)
    o = Oracle(p["W"], len(st["log"]) + p["T"] + len(st["log"]) + 16, purge_mode=1)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    out = o.tick(p["now"], p["tte"], [], [], [], [], [], p["T"])
    so = o.export()
    _check(digests(out["assign"], out["orphans"], out["evicted"], so["reg"], so["free"], so["hb"], so["queue"]),
           "oracle", fx)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_gpu_full_matches_reference(name):
    """The one-GPU HIP tick at configs[1]'s and configs[3]'s sizes against the reference
    captures."""
    from faasbal import GpuBalancer
    CFG = dict(cfg1=CFG1, cfg3=CFG3)[name]
    p, st = _cfg2_state(CFG)
    g = GpuBalancer(p["W"], 2 * len(st["log"]) + p["T"] + 16, max_events=1, device=0)
    g.load(st)
    out = g.tick(p["now"], p["tte"], n_pending=p["T"])
    sg = g.read_state(with_log=False)
    assert out["result"]["n_assigned"] == CFG["n_assigned"]
    _check(digests(out["assign"], out["orphans"], out["evicted"], sg["reg"], sg["free"], sg["hb"], sg["queue"]),
           "HIP tick", CFG)
    g.close()


def _cmp(a, b, t):
    for k in ("reconnect", "assign", "orphans", "evicted"):
        np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d %s" % (t, k))


@pytest.mark.gpu
@pytest.mark.parametrize("window,eager,resident", [(-1, False, False), (0, False, False), (-1, True, True)],
                         ids=["auto", "general", "eager-resident"])
def test_gpu_stream_1m_workers_matches_oracle(window, eager, resident):
    """configs[4] per GPU: 1M workers, 64K new tasks + 64K results + joins +
    heartbeats per tick, the clock advancing so silent workers expire; committed
    ticks, every output and the post-state compared with the oracle (heap purge).
    auto: level-0 ticks after the first run as window ticks; general:
    every tick on the general path (fb_set_window(0)); eager-resident: as bench.py's
    stream value runs it -- message batches in HBM, window commits enqueued behind
    their ticks (fb_set_eager_commit)."""
    from faasbal import GpuBalancer
    from oracle import Oracle
    W, T = 1 << 20, 65536
    st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
    # 50 ms per tick: workers whose last heartbeat is 9.8+ s old expire along the way
    ticks = synth.stream_ticks(st, n_ticks=4, seed=2, tasks_per_tick=T, results_per_tick=T, dt=0.05)
    cap = len(st["log"]) + 8 * T
    E = max(len(t["ev_kind"]) for t in ticks)
    g = GpuBalancer(W, cap, max_events=E, device=0)
    g.set_window(window)
    g.set_eager_commit(eager)
    g.load(st)
    o = Oracle(W, cap, purge_mode=2)  # heap purge: per-event clocks over 1M slots
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    carried, n_orph = 0, 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        if resident:
            import torch
            dev = [torch.from_numpy(np.ascontiguousarray(tk[k])).to("cuda:0")
                   for k in ("ev_kind", "ev_slot", "ev_val", "ev_ts", "ev_seq")]
            g.stage_device(tk["now"], *dev)
            g.launch_staged(10.0, n)
            r = g.wait()
            a = dict(result=r, reconnect=g.event_status(), assign=g.assignments(), orphans=g.orphans(),
                     evicted=g.evicted())
            g.commit()
            del dev
        else:
            a = g.tick(*args)
        b = o.tick(*args)
        _cmp(a, b, t)
        assert len(b["assign"]) > 0, "the stream must dispatch"
        n_orph += len(b["orphans"])
        carried = n + len(b["orphans"]) - len(b["assign"])
    assert n_orph > 0, "silent workers must expire and their tasks be redistributed"
    sg, so = g.read_state(), o.export()
    for k in ("reg", "queue", "log"):
        np.testing.assert_array_equal(sg[k], so[k], err_msg=k)
    m = so["reg"].astype(bool)
    np.testing.assert_array_equal(sg["free"][m], so["free"][m])
    np.testing.assert_array_equal(sg["hb"][m], so["hb"][m])
    wt, _ = g.window_stats()
    assert (wt >= 2) if window else (wt == 0), "window ticks: %d" % wt
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,xself,xcfirst", [(2, 1, 1), (4, 1, 1), (8, 1, 1), (4, 0, 1), (2, 1, 0)])
def test_gpu_sharded_16m_x_1m_matches_oracle(world, xself, xcfirst, monkeypatch):
    """configs[3]: 16M pending tasks x 1M workers, the worker table sharded by
    slot range over `world` rank contexts on one GPU; the exchange buffers are
    summed on the device (what the RCCL all-reduce computes).  xself 0: k_xscan's last
    workgroup prefixes the chunk totals (fb_set_path("xself", 0)) instead of phase 2's
    emission workgroups; xcfirst 0: phase 2's compaction workgroups after its queue
    workgroups in the grid (fb_set_path("xcfirst", 0))."""
    from faasbal.balancer import TEST_PATHS
    monkeypatch.setitem(TEST_PATHS, "xself", xself)
    monkeypatch.setitem(TEST_PATHS, "xcfirst", xcfirst)
    from test_gpu_sharded import _cmp as _cmp_sharded, _group, _group_tick
    W, T = 1 << 20, 16_000_000
    st = synth.zipf_state(W=W, seed=0)
    bals, o = _group(st, world, len(st["log"]) + T + len(st["log"]) + 16, max_events=1)
    merged, res = _group_tick(bals, 1000.0, 10.0, (), (), (), (), None, T)
    b = o.tick(1000.0, 10.0, [], [], [], [], [], T)
    assert len(b["assign"]) == res["n_assigned"] > 0 and len(b["orphans"]) > 0
    _cmp_sharded(bals, o, merged, b, 0)
    # ... and the merged decisions against the reference loop's own (cfg3_full_digests.json)
    import hashlib
    assert CFG3["params"]["W"] == W and CFG3["params"]["T"] == T
    for k, dt in (("assign", "<i4"), ("orphans", "<i8"), ("evicted", "<i4")):
        h = hashlib.sha256(np.asarray(merged[k], dt).tobytes()).hexdigest()
        assert h == CFG3["digests"][k]["sha256"], "sharded world %d: %s differs from the reference capture" % (world, k)
    for x in bals:
        x.close()


@pytest.mark.gpu
def test_gpu_sharded_stream_1m_workers_world8_matches_oracle():
    """configs[4] in its stated multi-GPU form: the 1M-worker table sharded by
    worker-id range over 8 rank contexts (one GPU; the exchange summed on the
    device, what the RCCL all-reduce computes), committed streaming ticks with
    64K new tasks, 64K results, joins and heartbeats each, silent workers
    expiring; every merged output and the reassembled state against the oracle
    (heap purge)."""
    from test_gpu_sharded import _cmp as _cmp_sharded, _group, _group_tick
    W, T, world = 1 << 20, 65536, 8
    st = synth.zipf_state(W=W, seed=0, dead_frac=0.0)
    ticks = synth.stream_ticks(st, n_ticks=3, seed=2, tasks_per_tick=T, results_per_tick=T, dt=0.05)
    E = max(len(t["ev_kind"]) for t in ticks)
    bals, o = _group(st, world, len(st["log"]) + 8 * T, max_events=E, purge_mode=2)
    carried, n_orph = 0, 0
    for t, tk in enumerate(ticks):
        n = carried + tk["n_new"]
        args = (tk["now"], 10.0, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], tk["ev_seq"], n)
        a, res = _group_tick(bals, *args)
        b = o.tick(*args)
        assert len(b["assign"]) > 0
        _cmp_sharded(bals, o, a, b, t)
        n_orph += len(b["orphans"])
        carried = n + len(b["orphans"]) - len(b["assign"])
    assert n_orph > 0, "silent workers must expire and their tasks be redistributed"
    for x in bals:
        x.close()
