"""Synthetic worker-pool states and event streams for the push balancer.

Everything here is seeded ``numpy.random.Generator(PCG64(seed))`` so the same
scenario is reproduced bit-for-bit here, on the GPU box and inside the golden
capture harness (``tests/golden/make_golden.py``).

State layout (host side, one entry per worker *slot*; the host maps a ZMQ
identity to a dense slot):

* ``reg``   u8   -- slot holds a live ``PushWorker`` record
                    (``task_dispatcher.py:203-207``)
* ``free``  i32  -- ``PushWorker.free_processes``
* ``hb``    f64  -- ``PushWorker.last_heartbeat``
* ``epoch`` u32  -- first in-flight-log sequence number owned by the current
                    registration (build-defined, needed for redistribution)
* ``queue`` i32  -- the ``free_workers`` OrderedDict of
                    ``start_heartbeat`` (``task_dispatcher.py:327``) in LRU order
* ``log``   i32  -- in-flight log: worker slot per dispatched task sequence
                    number, -1 once completed.

Event kinds mirror the message types handled at ``task_dispatcher.py:347-387``.
"""
from __future__ import annotations

import numpy as np

EV_REGISTER = 0
EV_RECONNECT = 1
EV_HEARTBEAT = 2
EV_RESULT = 3
EV_OTHER = 4
EV_NAMES = ("register", "reconnect", "heartbeat", "result", "ready")


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def empty_tick(now, n_new=0):
    return dict(now=float(now), n_new=int(n_new),
                ev_kind=np.zeros(0, np.uint8), ev_slot=np.zeros(0, np.int32),
                ev_val=np.zeros(0, np.int32), ev_ts=np.zeros(0, np.float64),
                ev_pick=np.zeros(0, np.uint32), ev_seq=np.full(0, -1, np.int64))


def random_scenario(seed, W=24, n_ticks=4, max_events=30, max_new=60,
                    tte=10.0, t0=1000.0, with_log=True):
    """Small adversarial scenario: re-register with 0/-1 processes, reconnects,
    late results, unknown ids, deaths and exact ``now - hb == tte`` boundaries
    (all times are multiples of 0.25 so the fp64 subtraction is exact)."""
    rng = _rng(seed)
    reg = rng.random(W) < 0.6
    free = np.where(reg, rng.integers(-1, 6, W), 0).astype(np.int32)
    hb = np.where(reg, t0 - 0.25 * rng.integers(0, 56, W), 0.0)
    cand = [s for s in range(W) if reg[s] and (
        (free[s] > 0 and rng.random() < 0.9) or (free[s] <= 0 and rng.random() < 0.2))]
    queue = rng.permutation(np.asarray(cand, np.int32)) if cand else np.zeros(0, np.int32)
    log = []
    if with_log:
        for s in range(W):
            if reg[s]:
                log += [s] * int(rng.integers(0, 4))
        # completed entries and stale entries of unregistered slots (inert)
        log += [-1] * int(rng.integers(0, 4))
        unreg = [s for s in range(W) if not reg[s]]
        if unreg:
            log += list(rng.choice(unreg, size=int(rng.integers(0, 3))))
        log = list(rng.permutation(np.asarray(log, np.int32))) if log else []
    ticks = []
    now = t0
    for _ in range(n_ticks):
        prev = now
        if rng.random() < 0.3:
            now = prev + 0.25 * int(rng.integers(30, 60))
        else:
            now = prev + 0.25 * int(rng.integers(0, 24))
        E = int(rng.integers(0, max_events + 1))
        span = int(round((now - prev) / 0.25))
        ts = np.sort(prev + 0.25 * rng.integers(0, span + 1, E)).astype(np.float64)
        kind = rng.choice(5, size=E, p=[0.15, 0.12, 0.3, 0.38, 0.05]).astype(np.uint8)
        # bias events towards a subset of slots so some slots see several events
        hot = rng.integers(0, W, max(1, W // 3))
        slot = np.where(rng.random(E) < 0.5, rng.choice(hot, E), rng.integers(0, W, E)).astype(np.int32)
        val = rng.integers(-1, 7, E).astype(np.int32)
        pick = rng.integers(0, 2 ** 31, E).astype(np.uint32)
        ticks.append(dict(now=float(now), n_new=int(rng.integers(0, max_new + 1)),
                          ev_kind=kind, ev_slot=slot, ev_val=val, ev_ts=ts,
                          ev_pick=pick, ev_seq=np.full(E, -1, np.int64)))
    return dict(W=W, tte=float(tte), t0=float(t0),
                init_reg=reg.astype(np.uint8), init_free=free, init_hb=hb.astype(np.float64),
                init_epoch=np.zeros(W, np.uint32),
                init_queue=np.asarray(queue, np.int32), init_log=np.asarray(log, np.int32),
                ticks=ticks)


def random_deque_scenario(seed, W=24, n_ticks=4, max_events=30, max_new=60, t0=1000.0, dup_frac=0.3):
    """Small adversarial scenario for the loop without heartbeats,
    ``PushDispatcher.start`` (``task_dispatcher.py:251-322``): the deque holds
    some ids several times (repeated registers), registers with 0/-1 processes,
    results that bring a worker back to 1 free process, and message kinds
    start() ignores.  Results only come from ids with a record (another id's
    result raises KeyError in the reference, :291)."""
    rng = _rng(seed + 7919)
    reg = rng.random(W) < 0.6
    free = np.where(reg, rng.integers(-1, 6, W), 0).astype(np.int32)
    hb = np.where(reg, t0 - 0.25 * rng.integers(0, 56, W), 0.0)
    tok = [s for s in range(W) if reg[s] and (free[s] > 0 and rng.random() < 0.9 or rng.random() < 0.15)]
    if tok:
        tok += list(rng.choice(tok, size=int(rng.integers(0, int(dup_frac * len(tok)) + 2))))
    queue = rng.permutation(np.asarray(tok, np.int32)) if tok else np.zeros(0, np.int32)
    log = []
    for s in range(W):
        if reg[s]:
            log += [s] * int(rng.integers(0, 4))
    log += [-1] * int(rng.integers(0, 4))
    log = list(rng.permutation(np.asarray(log, np.int32))) if log else []
    known = set(np.nonzero(reg)[0].tolist())
    ticks = []
    now = t0
    for _ in range(n_ticks):
        prev = now
        now = prev + 0.25 * int(rng.integers(0, 24))
        E = int(rng.integers(0, max_events + 1))
        ts = np.sort(prev + 0.25 * rng.integers(0, int(round((now - prev) / 0.25)) + 1, E)).astype(np.float64)
        kind = rng.choice(5, size=E, p=[0.25, 0.08, 0.1, 0.5, 0.07]).astype(np.uint8)
        hot = rng.integers(0, W, max(1, W // 4))
        slot = np.where(rng.random(E) < 0.6, rng.choice(hot, E), rng.integers(0, W, E)).astype(np.int32)
        val = rng.integers(-1, 6, E).astype(np.int32)
        for i in range(E):
            if kind[i] == EV_REGISTER:
                known.add(int(slot[i]))
            elif kind[i] == EV_RESULT and int(slot[i]) not in known:
                kind[i] = EV_HEARTBEAT  # start() ignores it
        ticks.append(dict(now=float(now), n_new=int(rng.integers(0, max_new + 1)),
                          ev_kind=kind, ev_slot=slot, ev_val=val, ev_ts=ts,
                          ev_pick=rng.integers(0, 2 ** 31, E).astype(np.uint32),
                          ev_seq=np.full(E, -1, np.int64)))
    return dict(W=W, tte=float("inf"), t0=float(t0),
                init_reg=reg.astype(np.uint8), init_free=free, init_hb=hb.astype(np.float64),
                init_epoch=np.zeros(W, np.uint32),
                init_queue=np.asarray(queue, np.int32), init_log=np.asarray(log, np.int32),
                ticks=ticks)


def zipf_deque_state(W=65536, seed=0, now=1000.0, cap=32, zipf_a=1.5, dup_frac=0.0):
    """Config-3 loads for the loop without heartbeats (start(), :251-322): no
    deaths; the deque holds every worker with free > 0 once, plus ``dup_frac``
    of them a second time (re-registered while queued)."""
    st = zipf_state(W=W, seed=seed, now=now, cap=cap, dead_frac=0.0, zipf_a=zipf_a)
    if dup_frac > 0:
        rng = _rng(seed + 104729)
        q = st["queue"]
        dup = rng.choice(q, size=int(dup_frac * len(q)), replace=False)
        pos = np.sort(rng.integers(0, len(q) + 1, len(dup)))
        st["queue"] = np.insert(q, pos, dup).astype(np.int32)
    return st


def uniform_state(W=1000, seed=0, now=1000.0, cap=256):
    """Config 2 (BASELINE.json configs[1]): every worker cap 256, busy ~ U[0,128),
    no deaths (hb = now - U[0, 9.9)), random LRU permutation."""
    rng = _rng(seed)
    busy = rng.integers(0, 128, W)
    free = (cap - busy).astype(np.int32)
    hb = now - rng.uniform(0.0, 9.9, W)
    queue = rng.permutation(W).astype(np.int32)
    return dict(W=W, reg=np.ones(W, np.uint8), free=free, hb=hb.astype(np.float64),
                epoch=np.zeros(W, np.uint32), queue=queue, log=np.zeros(0, np.int32))


def zipf_state(W=65536, seed=0, now=1000.0, cap=32, dead_frac=0.05, zipf_a=1.5):
    """Config 3 (BASELINE.json configs[2]): cap 32, busy = min(Zipf(1.5)-1, 32),
    5 % of workers with hb = now - 10.5 (dead at tte = 10), the rest
    now - U[0, 9.9); in-flight log holds ``busy`` tasks per worker in random
    dispatch order; LRU queue = random permutation of workers with free > 0."""
    rng = _rng(seed)
    busy = np.minimum(rng.zipf(zipf_a, W) - 1, cap)
    free = (cap - busy).astype(np.int32)
    hb = now - rng.uniform(0.0, 9.9, W)
    dead = rng.permutation(W)[: int(round(dead_frac * W))]
    hb[dead] = now - 10.5
    queued = np.nonzero(free > 0)[0]
    queue = rng.permutation(queued).astype(np.int32)
    log = np.repeat(np.arange(W, dtype=np.int32), busy)
    log = rng.permutation(log).astype(np.int32)
    return dict(W=W, reg=np.ones(W, np.uint8), free=free, hb=hb.astype(np.float64),
                epoch=np.zeros(W, np.uint32), queue=queue, log=log)


def state_to_scenario(st, ticks, tte=10.0):
    return dict(W=int(st["W"]), tte=float(tte), t0=float(ticks[0]["now"]) if ticks else 0.0,
                init_reg=st["reg"], init_free=st["free"], init_hb=st["hb"],
                init_epoch=st["epoch"], init_queue=st["queue"], init_log=st["log"],
                ticks=ticks)


def churn_ticks(st, n_ticks, seed=2, tasks_per_tick=1024, join_frac=0.001,
                expire_frac=0.001, results_per_tick=512, now0=1000.0, dt=1.0):
    """Config 5 shape at small scale: per tick joins (register), expiries (the
    worker stops heart-beating) and result events on in-flight tasks.  Result
    events carry ``ev_pick``; the driver resolves them to a concrete in-flight
    sequence number at run time."""
    rng = _rng(seed)
    W = int(st["W"])
    ticks = []
    now = now0
    silent = np.zeros(W, bool)
    for _ in range(n_ticks):
        prev = now
        now = prev + dt
        nj = max(1, int(join_frac * W))
        ne = max(1, int(expire_frac * W))
        silent[rng.integers(0, W, ne)] = True
        joins = rng.integers(0, W, nj)
        alive = np.nonzero(~silent)[0]
        hbs = rng.choice(alive, size=min(len(alive), W // 8), replace=False) if len(alive) else np.zeros(0, int)
        res = rng.choice(alive, size=results_per_tick) if len(alive) else np.zeros(0, int)
        kinds = np.concatenate([np.full(nj, EV_REGISTER), np.full(len(hbs), EV_HEARTBEAT),
                                np.full(len(res), EV_RESULT)]).astype(np.uint8)
        slots = np.concatenate([joins, hbs, res]).astype(np.int32)
        vals = np.concatenate([rng.integers(1, 33, nj), np.zeros(len(hbs) + len(res), int)]).astype(np.int32)
        order = rng.permutation(len(kinds))
        E = len(kinds)
        ts = np.sort(prev + (now - prev) * rng.random(E))
        ticks.append(dict(now=float(now), n_new=int(tasks_per_tick), ev_kind=kinds[order],
                          ev_slot=slots[order], ev_val=vals[order], ev_ts=ts,
                          ev_pick=rng.integers(0, 2 ** 31, E).astype(np.uint32),
                          ev_seq=np.full(E, -1, np.int64)))
    return ticks


def stream_ticks(st, n_ticks, seed=2, tasks_per_tick=65536, results_per_tick=65536, join_frac=0.001,
                 hb_frac=0.01, now0=1000.0, dt=0.01):
    """Config 5 (BASELINE.json configs[4]) per GPU: every tick ``tasks_per_tick``
    new tasks, ``results_per_tick`` results of distinct in-flight tasks of the
    initial log (their ``ev_seq`` resolved here, so no host model of the GPU's
    assignments is needed), ``join_frac`` re-registrations and ``hb_frac``
    heartbeats; the clock advances ``dt`` per tick, so workers that send
    nothing age towards the timeout and die (churn)."""
    rng = _rng(seed)
    W = int(st["W"])
    log = st["log"]
    inflight = np.nonzero(log >= 0)[0]
    order = rng.permutation(inflight)
    need = n_ticks * results_per_tick
    if need > len(order):
        raise ValueError("initial log holds %d in-flight tasks, %d results requested" % (len(order), need))
    ticks = []
    now = now0
    nj, nh = max(1, int(join_frac * W)), max(1, int(hb_frac * W))
    for t in range(n_ticks):
        prev = now
        now = prev + dt
        seq = order[t * results_per_tick:(t + 1) * results_per_tick].astype(np.int64)
        joins = rng.integers(0, W, nj)
        hbs = rng.integers(0, W, nh)
        kinds = np.concatenate([np.full(nj, EV_REGISTER), np.full(nh, EV_HEARTBEAT),
                                np.full(len(seq), EV_RESULT)]).astype(np.uint8)
        slots = np.concatenate([joins, hbs, log[seq]]).astype(np.int32)
        vals = np.concatenate([rng.integers(1, 33, nj), np.zeros(nh + len(seq), int)]).astype(np.int32)
        seqs = np.concatenate([np.full(nj + nh, -1, np.int64), seq])
        perm = rng.permutation(len(kinds))
        E = len(kinds)
        ts = np.sort(prev + dt * rng.random(E))
        ticks.append(dict(now=float(now), n_new=int(tasks_per_tick), ev_kind=kinds[perm], ev_slot=slots[perm],
                          ev_val=vals[perm], ev_ts=ts, ev_seq=seqs[perm]))
    return ticks
