"""Capture golden vectors from the REFERENCE push dispatcher (run here only).

This script imports ``/root/reference/task_dispatcher.py`` unmodified, with stub
``zmq``/``redis`` modules, a frozen controllable clock and fake socket / poller /
pub-sub / redis objects (recipe: SURVEY.md Appendix B), and drives the
reference's own ``PushDispatcher.start_heartbeat`` loop
(``task_dispatcher.py:324-419``) through scripted ticks:

* for every inbound event i of a tick: one iteration with nothing inbound at
  clock ``ts_i`` (the reference purges at ts_i, ``:390``), then one iteration
  delivering the event at ``ts_i`` (``:343-387``);  pub/sub tasks are hidden
  during this phase (a legal arrival order for the reference);
* then the dispatch phase at clock ``now``: one task per iteration via
  ``get_message`` (``:393-419``) until the tick's tasks run out or the LRU queue
  is empty.

The build-defined redistribution is replayed through the
same loop: at the first ``get_message`` of the dispatch phase, tasks in flight on
registrations that died during the tick are put, in ascending original dispatch
sequence, ahead of the pending tasks.

Only data leaves this script: ``tests/golden/*.npz`` (inputs + expected outputs).
No reference source is copied.  Usage:  python tests/golden/make_golden.py [all|heartbeat|deque|cfg1full|cfg2full|cfg3full]

The same harness drives the loop without heartbeats, ``PushDispatcher.start``
(``task_dispatcher.py:251-322``, a deque of ids instead of the OrderedDict) for
the ``deque_*.npz`` vectors.
"""
from __future__ import annotations

import collections
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
from faasbal import synth  # noqa: E402

REF_DIR = "/root/reference"


def load_reference():
    sys.dont_write_bytecode = True
    zmq = types.ModuleType("zmq")
    zmq.ROUTER, zmq.REP, zmq.DEALER, zmq.POLLIN = 6, 4, 5, 1

    class Poller:
        def register(self, *a, **k):
            pass
    zmq.Poller = Poller
    sys.modules["zmq"] = zmq
    sys.modules["redis"] = types.ModuleType("redis")
    cwd = os.getcwd()
    sys.path.insert(0, REF_DIR)
    try:
        import task_dispatcher as td  # noqa: F401
    finally:
        os.chdir(cwd)  # the reference chdirs at import (task_dispatcher.py:16)
        sys.path.remove(REF_DIR)
    return td


class _Wire:
    """Stands in for a serialized payload: ``.encode()``/``.decode()`` return it."""
    __slots__ = ("obj",)

    def __init__(self, obj):
        self.obj = obj

    def encode(self, *a):
        return self

    def decode(self, *a):
        return self


class _Stop(Exception):
    pass


def wid(slot):
    return b"w%06d" % slot


def slot_of(w):
    return int(w[1:])


class RefHarness:
    """Drives the reference loop; also acts as its socket, poller, subscriber
    and redis client."""

    def __init__(self, td, scen, purge_once=False, loop="start_heartbeat"):
        self.td = td
        self.loop = loop
        self.scen = scen
        self.clock = [float(scen.get("t0", 0.0))]
        td.time = types.SimpleNamespace(time=lambda: self.clock[0])
        td.serialize = lambda obj: _Wire(obj)
        td.deserialize = lambda w: w.obj
        W = int(scen["W"])
        self.W = W
        tte = scen["tte"]
        if loop == "start":
            # PushDispatcher.start keeps a collections.deque (:254) that may repeat ids
            self.queue = collections.deque(wid(int(s)) for s in scen["init_queue"])
            td.deque = lambda: self.queue
        else:
            q = collections.OrderedDict()
            for s in scen["init_queue"]:
                q[wid(int(s))] = None
            self.queue = q
            td.OrderedDict = lambda: self.queue
        d = td.PushDispatcher.__new__(td.PushDispatcher)
        d.workers = {}
        d.time_to_expire = tte
        d.socket = self
        d.poller = self
        d.subscriber = self
        d.redis_client = self
        for s in range(W):
            if scen["init_reg"][s]:
                pw = td.PushDispatcher.PushWorker(tte)
                pw.free_processes = int(scen["init_free"][s])
                pw.last_heartbeat = float(scen["init_hb"][s])
                d.workers[wid(s)] = pw
        self.d = d
        if purge_once:
            orig = d.purge_workers
            self._purge_key = None

            def purge_once_wrapper(fw):
                key = (self.clock[0], self._event_epoch)
                if key == self._purge_key:
                    return
                orig(fw)
                self._purge_key = key
            d.purge_workers = purge_once_wrapper
        self._event_epoch = 0
        # purge-once runs: the worker set changes only when a purge actually ran or an
        # event was delivered, so the O(W) key sync is skipped otherwise (a 1M-task
        # dispatch phase over 64K workers stays O(T), not O(T * W))
        self._dirty = True
        self._purge_once = purge_once
        if purge_once:
            orig2 = d.purge_workers

            def mark_dirty(fw):
                n = len(d.workers)
                orig2(fw)
                if len(d.workers) != n:
                    self._dirty = True
            d.purge_workers = mark_dirty
        # registration ids: bumped whenever a key (re)appears in d.workers
        self.regid = collections.defaultdict(int)
        self.keys = set(d.workers)
        for k in self.keys:
            self.regid[k] = 1
        # in-flight records: seq -> [wid, regid, state, task_id]
        self.records = []
        for s in scen["init_log"]:
            s = int(s)
            if s < 0:
                self.records.append([None, 0, "completed", "init"])
            elif scen["init_reg"][s] and scen["init_epoch"][s] == 0:
                self.records.append([wid(s), 1, "inflight", "init%d" % len(self.records)])
            else:
                self.records.append([wid(s), 0, "stale", "init%d" % len(self.records)])
        self.task_seq = {}
        self.ticks = scen["ticks"]
        self.t = -1
        self.out = []
        self.carried = []
        self._start_tick()

    # ------------------------------------------------------------------ ticks
    def _start_tick(self):
        self.t += 1
        if self.t >= len(self.ticks):
            raise _Stop()
        tk = self.ticks[self.t]
        self.tk = tk
        self.E = len(tk["ev_kind"])
        self.ev_i = 0
        self.stage = "pre" if self.E else "dispatch"
        self.seen = set(self.keys)
        self.died = set()
        self.reconnect = np.zeros(self.E, np.uint8)
        self.resolved_seq = np.full(self.E, -1, np.int64)
        self.assign = []
        self.orphans = None
        self.pending = None
        self.new_ids = ["t%d_%d" % (self.t, i) for i in range(int(tk["n_new"]))]
        self.gm_called = False
        self.gm_task = False
        self.sent_this_iter = []
        self.delivering = None
        self.first_dispatch = True

    def _sync_keys(self):
        cur = set(self.d.workers)
        for k in self.keys - cur:
            self.died.add((k, self.regid[k]))
        for k in cur - self.keys:
            self.regid[k] += 1
            self.seen.add(k)
        self.keys = cur

    def _compute_orphans(self):
        if self.orphans is not None:
            return
        self._sync_keys()
        orph = []
        for seq, rec in enumerate(self.records):
            if rec[2] == "inflight" and (rec[0], rec[1]) in self.died:
                orph.append(seq)
                rec[2] = "orphaned"
        self.orphans = orph
        # (a deque: taken from the front one task per loop iteration -- a list's pop(0)
        # made the 1M-task capture O(T^2) and a 16M-task one a matter of hours)
        self.pending = collections.deque([("orphan", seq) for seq in orph] + list(self.carried) +
                                         [("new", tid) for tid in self.new_ids])
        self.n_pending = len(self.pending)

    def _finish_iteration(self):
        # bookkeeping for the iteration that just ended
        if self.delivering is not None:
            i, w, kind, seq = self.delivering
            got_reconnect = any(dst == w and m.get("type") == "reconnect"
                                for dst, m in self.sent_this_iter)
            self.reconnect[i] = 1 if got_reconnect else 0
            if (not got_reconnect and kind == synth.EV_RESULT and seq >= 0
                    and self.records[seq][0] == w and self.records[seq][2] == "inflight"):
                self.records[seq][2] = "completed"
            self.delivering = None
        self.sent_this_iter = []
        if self._dirty or not self._purge_once:
            self._sync_keys()
            self._dirty = False

    def _end_tick(self):
        self._compute_orphans()
        carried = self.pending
        self.carried = carried
        evicted = sorted(slot_of(k) for k in self.seen - self.keys)
        post_reg = np.zeros(self.W, np.uint8)
        post_free = np.zeros(self.W, np.int64)
        post_hb = np.zeros(self.W, np.float64)
        for k, pw in self.d.workers.items():
            s = slot_of(k)
            post_reg[s] = 1
            post_free[s] = pw.free_processes
            post_hb[s] = pw.last_heartbeat
        self.out.append(dict(
            reconnect=self.reconnect, ev_seq=self.resolved_seq,
            assign=np.asarray(self.assign, np.int32),
            orphans=np.asarray(self.orphans, np.int64),
            evicted=np.asarray(evicted, np.int32), n_pending=self.n_pending,
            post_reg=post_reg, post_free=post_free, post_hb=post_hb,
            post_queue=np.asarray([slot_of(k) for k in self.queue], np.int32)))

    # --------------------------------------------------- poller / socket API
    def poll(self, timeout=None):
        self._finish_iteration()
        while True:
            if self.stage == "pre":
                self.clock[0] = float(self.tk["ev_ts"][self.ev_i])
                self.stage = "deliver"
                self.gm_called = False
                return []
            if self.stage == "deliver":
                self.clock[0] = float(self.tk["ev_ts"][self.ev_i])
                self.stage = "pre" if self.ev_i + 1 < self.E else "dispatch"
                self.gm_called = False
                return [(self, 1)]
            # dispatch phase
            if self.first_dispatch:
                self.first_dispatch = False
                self.clock[0] = float(self.tk["now"])
                self.gm_called = False
                self.gm_task = False
                return []
            if self.gm_called and self.gm_task:
                self.gm_called = False
                self.gm_task = False
                return []
            self._end_tick()
            self._start_tick()  # raises _Stop after the last tick

    def recv_multipart(self):
        i = self.ev_i
        self.ev_i += 1
        tk = self.tk
        kind = int(tk["ev_kind"][i])
        w = wid(int(tk["ev_slot"][i]))
        val = int(tk["ev_val"][i])
        seq = -1
        if kind == synth.EV_REGISTER:
            msg = {"type": "register", "data": {"num_processes": val}}
        elif kind == synth.EV_RECONNECT:
            msg = {"type": "reconnect", "data": {"free_processes": val}}
        elif kind == synth.EV_HEARTBEAT:
            msg = {"type": "heartbeat"}
        elif kind == synth.EV_RESULT:
            pick = int(tk["ev_pick"][i])
            infl = [q for q, r in enumerate(self.records) if r[0] == w and r[2] == "inflight"]
            if pick % 7 == 6 and self.records:
                seq = pick % len(self.records)
            elif pick % 5 != 4 and infl:
                seq = infl[pick % len(infl)]
            tid = self.records[seq][3] if seq >= 0 else "none"
            msg = {"type": "result", "data": {"task_id": tid, "status": "COMPLETED", "result": "r"}}
        else:
            msg = {"type": "ready"}
        self.resolved_seq[i] = seq
        self.delivering = (i, w, kind, seq)
        self._event_epoch += 1
        self._dirty = True
        return w, _Wire(msg)

    def send_multipart(self, parts):
        dst, payload = parts
        m = payload.obj
        self.sent_this_iter.append((dst, m))
        if m.get("type") == "task":
            tid = m["data"]["task_id"]
            assert tid == self._cur_task_id
            self.records.append([dst, self.regid[dst], "inflight", tid])
            self.assign.append(slot_of(dst))

    def get_message(self):
        self.gm_called = True
        if self.stage != "dispatch" or self.first_dispatch:
            return None
        self._compute_orphans()
        if not self.pending:
            self.gm_task = False
            return None
        kind, ref = self.pending.popleft()
        tid = self.records[ref][3] if kind == "orphan" else ref
        self._cur_task_id = tid
        self.gm_task = True
        return {"type": "message", "data": tid.encode()}

    def hget(self, key, field):
        return b"payload"

    def hset(self, key, mapping=None, **kw):
        pass

    def run(self):
        try:
            getattr(self.d, self.loop)()
        except _Stop:
            pass
        return self.out


# ---------------------------------------------------------------- fixtures
def pack(scen, outs, name, note):
    W = int(scen["W"])
    T = len(scen["ticks"])
    ev_off = np.cumsum([0] + [len(t["ev_kind"]) for t in scen["ticks"]]).astype(np.int64)
    cat = lambda key, dt: (np.concatenate([np.asarray(t[key], dt) for t in scen["ticks"]])
                           if T else np.zeros(0, dt))
    ocat = lambda key, dt: (np.concatenate([np.asarray(o[key], dt) for o in outs])
                            if outs else np.zeros(0, dt))
    ooff = lambda key: np.cumsum([0] + [len(o[key]) for o in outs]).astype(np.int64)
    arrs = dict(
        W=np.int64(W), tte=np.float64(scen["tte"]), n_ticks=np.int64(T),
        init_reg=scen["init_reg"].astype(np.uint8), init_free=scen["init_free"].astype(np.int32),
        init_hb=scen["init_hb"].astype(np.float64), init_epoch=scen["init_epoch"].astype(np.uint32),
        init_queue=scen["init_queue"].astype(np.int32), init_log=scen["init_log"].astype(np.int32),
        now=np.asarray([t["now"] for t in scen["ticks"]], np.float64),
        n_new=np.asarray([t["n_new"] for t in scen["ticks"]], np.int64),
        ev_off=ev_off, ev_kind=cat("ev_kind", np.uint8), ev_slot=cat("ev_slot", np.int32),
        ev_val=cat("ev_val", np.int32), ev_ts=cat("ev_ts", np.float64),
        ev_seq=ocat("ev_seq", np.int64),
        exp_reconnect=ocat("reconnect", np.uint8),
        exp_assign_off=ooff("assign"), exp_assign=ocat("assign", np.int32),
        exp_orphan_off=ooff("orphans"), exp_orphan=ocat("orphans", np.int64),
        exp_evicted_off=ooff("evicted"), exp_evicted=ocat("evicted", np.int32),
        exp_n_pending=np.asarray([o["n_pending"] for o in outs], np.int64),
        exp_post_reg=np.stack([o["post_reg"] for o in outs]) if outs else np.zeros((0, W), np.uint8),
        exp_post_free=np.stack([o["post_free"] for o in outs]).astype(np.int32) if outs else np.zeros((0, W), np.int32),
        exp_post_hb=np.stack([o["post_hb"] for o in outs]) if outs else np.zeros((0, W)),
        exp_post_queue_off=ooff("post_queue"), exp_post_queue=ocat("post_queue", np.int32),
        note=np.asarray(note),
    )
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    return path


def capture(td, scen, purge_once=False, loop="start_heartbeat"):
    return RefHarness(td, scen, purge_once=purge_once, loop=loop).run()


def digests(assign, orphans, evicted, post_reg, post_free, post_hb, post_queue):
    """sha256 of each output as little-endian bytes (post_free / post_hb of the
    registered slots only: the reference keeps no record for the others)."""
    import hashlib
    reg = np.asarray(post_reg, np.uint8)
    arrs = dict(assign=np.asarray(assign, "<i4"), orphans=np.asarray(orphans, "<i8"),
                evicted=np.asarray(evicted, "<i4"), post_reg=reg,
                post_free=np.asarray(post_free, np.int64)[reg == 1].astype("<i4"),
                post_hb=np.asarray(post_hb, "<f8")[reg == 1], post_queue=np.asarray(post_queue, "<i4"))
    return {k: {"sha256": hashlib.sha256(v.tobytes()).hexdigest(), "len": int(len(v))} for k, v in arrs.items()}


# BASELINE.json configs[2] at its stated size: the headline tick pinned against the
# reference itself (digests only: the outputs are MBs; tests recompute them)
CFG2_FULL = dict(W=65536, seed=0, T=1_000_000, now=1000.0, tte=10.0)
# ... and configs[3]'s one-GPU tick (16 M pending tasks x 1 M workers), the same way
CFG3_FULL = dict(W=1 << 20, seed=0, T=16_000_000, now=1000.0, tte=10.0)
# ... and configs[1] (100K tasks x 1K workers, uniform loads)
CFG1_FULL = dict(W=1000, seed=0, T=100_000, now=1000.0, tte=10.0, loads="uniform")


def cfg2_full_fixture(td, p=CFG2_FULL, name="cfg2_full_digests.json"):
    import json
    import time
    uniform = p.get("loads") == "uniform"
    st = (synth.uniform_state if uniform else synth.zipf_state)(W=p["W"], seed=p["seed"])
    scen = synth.state_to_scenario(st, [synth.empty_tick(p["now"], p["T"])], tte=p["tte"])
    t0 = time.perf_counter()
    o = capture(td, scen, purge_once=True)[0]
    dt = time.perf_counter() - t0
    out = dict(params=p, generator="faasbal.synth.%s(W, seed) + one tick of T pending tasks at now" % (
                   "uniform_state" if uniform else "zipf_state"),
               reference="task_dispatcher.py:324-419 via tests/golden/make_golden.py (purge once per unchanged "
                         "clock, SURVEY.md App. B), %.1f s in the capture container" % dt,
               n_assigned=int(len(o["assign"])), n_orphans=int(len(o["orphans"])),
               n_evicted=int(len(o["evicted"])), n_pending=int(o["n_pending"]),
               digests=digests(o["assign"], o["orphans"], o["evicted"], o["post_reg"], o["post_free"], o["post_hb"],
                               o["post_queue"]))
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    return [path]


def main(which="all"):
    td = load_reference()
    made = []
    if which in ("all", "heartbeat"):
        made += heartbeat_fixtures(td)
    if which in ("all", "deque"):
        made += deque_fixtures(td)
    if which in ("all", "cfg2full"):
        made += cfg2_full_fixture(td)
    if which in ("all", "cfg1full"):
        made += cfg2_full_fixture(td, CFG1_FULL, "cfg1_full_digests.json")
    if which == "cfg3full":  # (about an hour of reference loop; not part of "all")
        made += cfg2_full_fixture(td, CFG3_FULL, "cfg3_full_digests.json")
    for p in made:
        print(p, os.path.getsize(p))


def heartbeat_fixtures(td):
    made = []
    # 1) many small adversarial multi-tick scenarios, loop exactly as written
    for seed in range(48):
        W = [6, 12, 24, 48][seed % 4]
        scen = synth.random_scenario(seed, W=W, n_ticks=1 + seed % 6,
                                     max_events=[0, 8, 30, 80][(seed // 4) % 4],
                                     max_new=[0, 10, 60, 200][(seed // 2) % 4])
        outs = capture(td, scen)
        made.append(pack(scen, outs, "small_%02d" % seed,
                         "random_scenario seed=%d, reference loop as written" % seed))
    # 2) config-2 shape, reduced: uniform loads, W=1000, T=20000, one tick
    st = synth.uniform_state(W=1000, seed=0)
    scen = synth.state_to_scenario(st, [synth.empty_tick(1000.0, 20000)])
    made.append(pack(scen, capture(td, scen, purge_once=True), "cfg2_w1000_t20000",
                     "uniform_state(W=1000, seed=0), T=20000, purge once per unchanged clock"))
    # 3) config-3 shape, reduced: Zipf loads + 5% dead + in-flight log, W=4096, T=50000
    st = synth.zipf_state(W=4096, seed=0)
    scen = synth.state_to_scenario(st, [synth.empty_tick(1000.0, 50000)])
    made.append(pack(scen, capture(td, scen, purge_once=True), "cfg3_w4096_t50000",
                     "zipf_state(W=4096, seed=0), T=50000, purge once per unchanged clock"))
    # 4) config-5 shape, reduced: churn over several ticks
    st = synth.zipf_state(W=512, seed=3)
    ticks = synth.churn_ticks(st, n_ticks=14, seed=2, tasks_per_tick=600, join_frac=0.01,
                              expire_frac=0.01, results_per_tick=200)
    scen = synth.state_to_scenario(st, ticks)
    scen["t0"] = 1000.0
    made.append(pack(scen, capture(td, scen, purge_once=True), "cfg5_w512_churn",
                     "zipf_state(W=512, seed=3) + churn_ticks(14, seed=2), purge once per unchanged clock"))
    return made


def deque_fixtures(td):
    made = []
    # 5) the loop without heartbeats, PushDispatcher.start (:251-322): deque with
    #    repeated ids, registers with 0/-1, results bringing free back to 1
    for seed in range(24):
        W = [6, 12, 24, 48][seed % 4]
        scen = synth.random_deque_scenario(seed, W=W, n_ticks=1 + seed % 6,
                                           max_events=[0, 8, 30, 80][(seed // 4) % 4],
                                           max_new=[0, 10, 60, 200][(seed // 2) % 4])
        made.append(pack(scen, capture(td, scen, loop="start"), "deque_%02d" % seed,
                         "random_deque_scenario seed=%d, reference start() loop" % seed))
    st = synth.zipf_deque_state(W=2048, seed=4, dup_frac=0.05)
    scen = synth.state_to_scenario(st, [synth.empty_tick(1000.0, 30000)], tte=float("inf"))
    made.append(pack(scen, capture(td, scen, loop="start"), "deque_cfg3_w2048_t30000",
                     "zipf_deque_state(W=2048, seed=4, dup_frac=0.05), T=30000, reference start() loop"))
    return made


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "all")
