"""Sharded worker table (several ranks) vs the one-table oracle, on one GPU.

Every rank is a separate library context (its own slot range, log shard and
stream) in this process; the exchange all-reduce is a device-side SUM of the
ranks' exchange tensors -- the same reduction RCCL performs across GPUs.  The
merged outputs (assignments, orphans, evicted, reconnect flags) and the
reassembled state must equal the oracle's bit for bit.
"""
import numpy as np
import pytest

from faasbal import synth
from faasbal.balancer import TEST_PATHS
from oracle import Oracle

pytestmark = pytest.mark.gpu


def _group(st, world, log_cap, max_events=4096, purge_mode=1):
    import torch  # noqa: F401  (loads the HIP runtime before libfaasbal)
    from faasbal.sharded import ShardedBalancer

    W = len(st["reg"])
    bals = [ShardedBalancer(r, world, W, log_cap, max_events=max_events) for r in range(world)]
    for b in bals:
        b.load(st)
    o = Oracle(W, log_cap, purge_mode=purge_mode)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    return bals, o


def _group_tick(bals, *args, relaunches=None):
    import torch
    from faasbal import FaasbalError
    from faasbal._lib import FB_ERERUN
    from faasbal.sharded import merge_outputs

    for attempt in range(7):
        for b in bals:
            b.launch(*args)
        torch.cuda.synchronize()
        total = bals[0].exchange().clone()
        for b in bals[1:]:
            total += b.exchange()  # single contributor per byte: the uint8 sum is exact
        for b in bals:
            b.exchange().copy_(total)
        torch.cuda.synchronize()
        for b in bals:
            b.cont()
        res, codes = [], set()
        for b in bals:
            try:
                res.append(b.wait())
            except FaasbalError as e:
                codes.add(e.code)
        if not codes:
            break
        assert codes == {FB_ERERUN}, codes  # a relaunch is asked of every rank or of none
        assert not res
        if relaunches is not None:
            relaunches.append(attempt)
    for k in ("n_assigned", "n_orphans", "queue_len", "log_head", "fill_level"):
        assert len({r[k] for r in res}) == 1, k
    outs = []
    for b in bals:
        task, slot = b.local_assignments()
        assert np.all(np.diff(task) > 0)  # ascending global order in every log shard
        outs.append(dict(task=task, slot=slot, orphans=b.orphans(), evicted=b.evicted(), reconnect=b.event_status()))
    for b in bals[1:]:
        np.testing.assert_array_equal(outs[0]["reconnect"], b.event_status())
    merged = merge_outputs(outs, res[0]["n_assigned"])
    for b in bals:
        b.commit()
    return merged, res[0]


def _cmp(bals, o, a, b, t):
    for k in ("reconnect", "assign", "orphans", "evicted"):
        np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))
    so = o.export()
    reg = so["reg"].astype(bool)
    glog = np.full(len(so["log"]), -1, np.int32)
    for bal in bals:
        sg = bal.read_state()
        lo, hi = bal.base, bal.base + bal.n_local
        np.testing.assert_array_equal(sg["reg"], so["reg"][lo:hi], err_msg="tick %d reg" % t)
        m = reg[lo:hi]
        np.testing.assert_array_equal(sg["free"][m], so["free"][lo:hi][m], err_msg="tick %d free" % t)
        np.testing.assert_array_equal(sg["hb"][m], so["hb"][lo:hi][m], err_msg="tick %d hb" % t)
        np.testing.assert_array_equal(sg["queue"], so["queue"], err_msg="tick %d queue" % t)
        assert sg["head"] == len(so["log"])
        glog[sg["log_seq"]] = sg["log"]
    np.testing.assert_array_equal(glog, so["log"], err_msg="tick %d log" % t)


@pytest.mark.parametrize("seed", range(12))
def test_sharded_random_multitick(seed):
    W = [37, 300, 1000][seed % 3]
    world = [2, 3, 4][(seed // 3) % 3]
    scen = synth.random_scenario(5000 + seed, W=W, n_ticks=5, max_events=[20, 200, 2000][seed % 3],
                                 max_new=[50, 400, 3000][(seed // 3) % 3])
    st = dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
              queue=scen["init_queue"], log=scen["init_log"])
    bals, o = _group(st, world, len(st["log"]) + 40000)
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
        a, _ = _group_tick(bals, *args)
        b = o.tick(*args)
        _cmp(bals, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_config3(world):
    """BASELINE configs[2] table split over ranks: 1M tasks x 64K workers."""
    st = synth.zipf_state(W=65536, seed=0)
    T = 1_000_000
    bals, o = _group(st, world, len(st["log"]) + T + len(st["log"]) + 16)
    a, r = _group_tick(bals, 1000.0, 10.0, [], [], [], [], [], T)
    b = o.tick(1000.0, 10.0, [], [], [], [], [], T)
    assert r["n_orphans"] > 0
    _cmp(bals, o, a, b, 0)


def test_sharded_churn():
    st = synth.zipf_state(W=65536, seed=3)
    ticks = synth.churn_ticks(st, n_ticks=3, seed=2, tasks_per_tick=65536, join_frac=0.001, expire_frac=0.001,
                              results_per_tick=8192)
    bals, o = _group(st, 2, len(st["log"]) + 3 * 65536 + 200_000, max_events=20000)
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
        a, _ = _group_tick(bals, *args)
        b = o.tick(*args)
        _cmp(bals, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


def test_sharded_world1_equals_one_gpu():
    st = synth.zipf_state(W=4096, seed=9)
    bals, o = _group(st, 1, len(st["log"]) * 2 + 100_000)
    a, _ = _group_tick(bals, 1000.0, 10.0, [], [], [], [], [], 60_000)
    b = o.tick(1000.0, 10.0, [], [], [], [], [], 60_000)
    _cmp(bals, o, a, b, 0)


@pytest.fixture
def logscan(monkeypatch):
    """Phase 1's log role through k_logscan (the default past 128K local slots)."""
    monkeypatch.setitem(TEST_PATHS, "logscan", 1)


@pytest.mark.parametrize("seed", range(6))
def test_sharded_random_multitick_logscan(logscan, seed):
    test_sharded_random_multitick(seed)


def test_sharded_churn_logscan(logscan):
    test_sharded_churn()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_wide_sort_digits(world):
    """A 18-bit global slot space: every rank sorts the whole message batch by
    global slot with two passes of 9-bit digits, then applies its own range."""
    W, E = (1 << 17) + 5, 6000
    rng = np.random.default_rng(world)
    st = synth.zipf_state(W=W, seed=world, dead_frac=0.02)
    bals, o = _group(st, world, 2 * len(st["log"]) + 100_000, max_events=E)
    slot = rng.integers(0, W, E).astype(np.int32)
    kind = rng.choice([synth.EV_REGISTER, synth.EV_HEARTBEAT, synth.EV_RESULT, synth.EV_RECONNECT], size=E,
                      p=[0.1, 0.4, 0.4, 0.1]).astype(np.int32)
    val = rng.integers(0, 4, E).astype(np.int32)
    now = 1000.0
    ts = np.sort(now - rng.random(E)).astype(np.float64)
    args = (now, 10.0, kind, slot, val, ts, np.full(E, -1, np.int64), 20_000)
    a, _ = _group_tick(bals, *args)
    b = o.tick(*args)
    _cmp(bals, o, a, b, 0)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_wide_free_counts(world):
    """Free counts up to 10 000 (beyond the exchange byte and the 128-row round
    table): every round below the fill level is exact, so the sharded ticks match
    the oracle -- registrations with thousands of processes included."""
    rng = np.random.default_rng(40 + world)
    W, now = 600, 1000.0
    reg = np.ones(W, np.uint8)
    free = rng.integers(0, 10_001, W).astype(np.int32)
    hb = now - rng.random(W) * 9.9
    hb[rng.random(W) < 0.03] = now - 10.5
    queue = rng.permutation(np.nonzero(free > 0)[0]).astype(np.int32)
    log = rng.integers(-1, W, 20_000).astype(np.int32)
    st = dict(reg=reg, free=free, hb=hb, epoch=np.zeros(W, np.uint32), queue=queue, log=log)
    bals, o = _group(st, world, len(log) + 200_000, max_events=512)
    carried = 0
    for t in range(4):
        t_now = now + 0.5 * t
        E = 200
        kind = rng.choice([synth.EV_REGISTER, synth.EV_HEARTBEAT, synth.EV_RESULT, synth.EV_RECONNECT], size=E,
                          p=[0.2, 0.4, 0.3, 0.1]).astype(np.uint8)
        slot = rng.integers(0, W, E).astype(np.int32)
        val = rng.integers(0, 10_001, E).astype(np.int32)
        ts = np.sort(t_now - 0.5 * rng.random(E))
        n = carried + 25_000
        args = (t_now, 10.0, kind, slot, val, ts, np.full(E, -1, np.int64), n)
        a, r = _group_tick(bals, *args)
        b = o.tick(*args)
        assert o.export()["free"].max() > 255 and r["max_free"] == 255  # c travels clamped to a byte
        _cmp(bals, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_fill_level_beyond_128(world):
    """Fill levels of hundreds of rounds (600 workers with free counts up to 10 000,
    200 K tasks per tick): the sharded tick asks for a relaunch (FB_ERERUN) with a wider
    round table and two-byte exchanged counts, then matches the oracle; no FB_ERANGE."""
    rng = np.random.default_rng(70 + world)
    W, now = 600, 1000.0
    reg = np.ones(W, np.uint8)
    free = rng.integers(0, 10_001, W).astype(np.int32)
    hb = now - rng.random(W) * 9.9
    hb[rng.random(W) < 0.03] = now - 10.5
    queue = rng.permutation(np.nonzero(free > 0)[0]).astype(np.int32)
    log = rng.integers(-1, W, 20_000).astype(np.int32)
    st = dict(reg=reg, free=free, hb=hb, epoch=np.zeros(W, np.uint32), queue=queue, log=log)
    bals, o = _group(st, world, len(log) + 1_200_000, max_events=512)
    carried, levels, relaunches = 0, [], []
    for t in range(4):
        t_now = now + 0.5 * t
        E = 200
        kind = rng.choice([synth.EV_REGISTER, synth.EV_HEARTBEAT, synth.EV_RESULT, synth.EV_RECONNECT], size=E,
                          p=[0.2, 0.4, 0.3, 0.1]).astype(np.uint8)
        slot = rng.integers(0, W, E).astype(np.int32)
        val = rng.integers(0, 10_001, E).astype(np.int32)
        ts = np.sort(t_now - 0.5 * rng.random(E))
        n = carried + 200_000
        args = (t_now, 10.0, kind, slot, val, ts, np.full(E, -1, np.int64), n)
        a, r = _group_tick(bals, *args, relaunches=relaunches)
        b = o.tick(*args)
        levels.append(r["fill_level"])
        _cmp(bals, o, a, b, t)
        carried = n + len(b["orphans"]) - len(b["assign"])
    assert max(levels) > 128, levels
    assert relaunches, "the first wide tick must ask for a relaunch"


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_wide_table_with_tight_log_shards(world):
    """A narrow first launch cannot know N_eff (free counts beyond its round table), so
    its log check would see the whole backlog: more pending tasks (1.5 M) than the
    ranks' capacity (~0.9 M) and log shards sized for the capacity, not the backlog.
    Every rank must ask for the relaunch (FB_ERERUN before FB_ENOSPC), and
    the wide relaunch fits and matches the oracle."""
    import torch  # noqa: F401
    from faasbal.sharded import ShardedBalancer
    rng = np.random.default_rng(90 + world)
    W, now = 600, 1000.0
    reg = np.ones(W, np.uint8)
    free = rng.integers(0, 3001, W).astype(np.int32)
    hb = now - rng.random(W) * 9.9
    queue = rng.permutation(np.nonzero(free > 0)[0]).astype(np.int32)
    log = rng.integers(-1, W, 20_000).astype(np.int32)
    st = dict(reg=reg, free=free, hb=hb, epoch=np.zeros(W, np.uint32), queue=queue, log=log)
    T = 1_500_000
    cap_sum = int(free[queue].sum())
    assert cap_sum < 1_000_000 < T
    rank_cap = len(log) + 1_100_000  # > the capacity any rank can take, < the backlog
    bals = [ShardedBalancer(r, world, W, rank_cap, max_events=16) for r in range(world)]
    for b in bals:
        b.load(st)
    o = Oracle(W, len(log) + T + 16, purge_mode=1)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    relaunches = []
    a, r = _group_tick(bals, now, 10.0, [], [], [], [], [], T, relaunches=relaunches)
    b = o.tick(now, 10.0, [], [], [], [], [], T)
    assert relaunches and r["n_assigned"] == cap_sum and r["fill_level"] > 128
    _cmp(bals, o, a, b, 0)
    for x in bals:
        x.close()


@pytest.mark.parametrize("world,nbq,cap", [(3, 1, 30), (3, 17, 30), (3, 256, 30), (3, 257, 30), (3, 17, 60),
                                           (3, 256, 120), (2, 40, 120), (16, 17, 30)])
def test_sharded_exchanged_rows_shapes(world, nbq, cap):
    """Phase 2 from the exchanged block rows (<= 256 queue blocks, <= 16 ranks) and, at a
    32-row table, group rows (16 blocks per group, a partial last group): queue lengths
    around those limits (257 blocks: the phase-2 scan instead), tables of 32 / 64 / 128
    rows (the second tick sizes its table from the first's max free count), 16 ranks."""
    rng = np.random.default_rng(1000 * nbq + cap + world)
    W = max(world, nbq * 256 - 10)
    now = 1000.0
    free = rng.integers(0, cap + 1, W).astype(np.int32)
    hb = np.where(rng.random(W) < 0.05, now - 10.5, now - rng.random(W) * 9.0)
    queue = rng.permutation(np.nonzero(free > 0)[0]).astype(np.int32)
    if len(queue) < W - 12:  # fill the queue to the target length with free-0 workers (c = 1)
        rest = np.setdiff1d(np.arange(W), queue)[: W - 12 - len(queue)]
        queue = rng.permutation(np.concatenate([queue, rest])).astype(np.int32)
    log = rng.integers(-1, W, 3 * W).astype(np.int32)
    st = dict(reg=np.ones(W, np.uint8), free=free, hb=hb, epoch=np.zeros(W, np.uint32), queue=queue, log=log)
    n_new = max(1, int(W * cap / 8))
    bals, o = _group(st, world, len(log) + 4 * n_new + W + 16, max_events=64)
    carried = 0
    for t in range(3):
        args = (now + 0.1 * t, 10.0, [], [], [], [], [], carried + n_new)
        a, r = _group_tick(bals, *args)
        b = o.tick(*args)
        _cmp(bals, o, a, b, t)
        carried = carried + n_new + len(b["orphans"]) - len(b["assign"])


def test_sharded_length_check_failure_aborts_the_group():
    """A device-reported length that fails fb_tick_wait's check on ONE rank (injected
    there) fails the group's tick: LocalShardGroup commits no rank, so the shards stay in
    step and the same tick then runs against the oracle as if the failure never happened
    (DistShardGroup settles the same way: commit only when every rank succeeded)."""
    import torch  # noqa: F401
    from faasbal import FaasbalError
    from faasbal.sharded import LocalShardGroup

    st = synth.zipf_state(W=4096, seed=4)
    T = 30_000
    grp = LocalShardGroup(3, 4096, len(st["log"]) + 4 * T + 16, max_events=64)
    grp.load(st)
    o = Oracle(4096, len(st["log"]) + 4 * T + 16)
    o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
    grp.bals[1].set_path("fault_qlen", 1 << 30)
    args = (1000.0, 10.0, [synth.EV_HEARTBEAT], [7], [0], [999.0], [-1], T)
    with pytest.raises(FaasbalError, match="queue length"):
        grp.tick(*args)
    for t in range(2):
        a = grp.tick(*args)
        b = o.tick(*args)
        for k in ("reconnect", "assign", "orphans", "evicted"):
            np.testing.assert_array_equal(a[k], b[k], err_msg="tick %d: %s" % (t, k))
        args = (1001.0, 10.0, [], [], [], [], [], T // 3)
    np.testing.assert_array_equal(grp.read_state()["queue"], o.export()["queue"])
