"""GpuPushDispatcher end to end: the reference-captured golden ticks replayed as
real ZMQ-style messages (dill+base64 frames) through fake socket / poller /
pub-sub / Redis objects.  Checks, per tick, every message the dispatcher sends
(``reconnect`` replies, then ``task`` messages with their task ids and target
identities), every Redis write, the LRU queue (as identities) and the worker
records -- against the expected outputs the reference loop produced
(tests/golden/*.npz, captured by tests/golden/make_golden.py)."""
import collections
import glob
import os

import numpy as np
import pytest

from faasbal import codec

GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if not os.path.basename(p).startswith("deque_"))  # start_heartbeat vectors
KIND_MSG = {0: "register", 1: "reconnect", 2: "heartbeat", 3: "result", 4: "ready"}


def wid(s):
    return b"w%06d" % int(s)


class FakePipe:
    """redis-py pipeline stand-in: commands queue up, ``execute`` runs them in order."""

    def __init__(self, env):
        self.env, self.cmds = env, []

    def hget(self, key, field):
        self.cmds.append(("hget", key, field))

    def hset(self, key, mapping=None):
        self.cmds.append(("hset", key, mapping))

    def execute(self):
        self.env.round_trips += 1
        out = []
        for op, key, arg in self.cmds:
            if op == "hget":
                out.append(("%s:%s" % (arg, key)).encode())
            else:
                self.env.hsets.append((key, dict(arg)))
                out.append(1)
        self.cmds = []
        return out


class FakeEnv:
    """ROUTER socket + poller + pub/sub + Redis client + clock, all in memory."""

    def __init__(self, pipelines=True):
        self.inbound = collections.deque()  # (identity, frame bytes, ts)
        self.tasks = collections.deque()
        self.sent = []
        self.hsets = []
        self.round_trips = 0
        if pipelines:
            self.pipeline = lambda transaction=True: FakePipe(self)
        self.now = 0.0
        self.t = 0.0
        self.sock = self
        self.redis = self
        self.sub = self

    # poller
    def poll(self, timeout=None):
        if self.inbound:
            return [(self, 1)]
        self.t = self.now  # inbound drained: the loop's clock moves to the tick's `now`
        return []

    # socket
    def recv_multipart(self):
        w, frame, ts = self.inbound.popleft()
        self.t = ts
        return [w, frame]

    def send_multipart(self, parts):
        self.sent.append((parts[0], codec.deserialize(parts[1].decode("utf-8"))))

    # pub/sub
    def get_message(self):
        if not self.tasks:
            return None
        return {"type": "message", "data": self.tasks.popleft().encode()}

    # redis
    def hget(self, key, field):
        self.round_trips += 1
        return ("%s:%s" % (field, key)).encode()

    def hset(self, key, mapping=None):
        self.round_trips += 1
        self.hsets.append((key, dict(mapping)))

    def clock(self):
        return self.t


def test_codec_matches_reference_format():
    msg = {"type": "result", "data": {"task_id": "t1", "status": "COMPLETED", "result": "x"}}
    s = codec.serialize(msg)
    assert isinstance(s, str) and s.endswith("\n")  # codecs base64 keeps line breaks
    assert codec.deserialize(s) == msg


@pytest.fixture(params=[pytest.param("gpu", marks=pytest.mark.gpu), "host"])
def dispatcher_cls(request, monkeypatch):
    """The real dispatcher on the GPU; on the CPU the same host logic over the
    oracle test double (tests/oracle_balancer.py) in place of libfaasbal."""
    import faasbal.dispatcher as D
    if request.param == "host":
        from oracle_balancer import OracleBalancer
        monkeypatch.setattr(D, "GpuBalancer", OracleBalancer)
    return D.GpuPushDispatcher


@pytest.fixture(params=[True, False], ids=["pipelined", "per-call"])
def pipelines(request):
    """Redis client with pipelines (batched host I/O) or without (one round trip per command)."""
    return request.param


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_dispatcher_replays_reference(path, dispatcher_cls, pipelines):
    GpuPushDispatcher = dispatcher_cls
    z = np.load(path)
    replay_golden(z, lambda sizes, env: GpuPushDispatcher(
        "127.0.0.1", 0, float(z["tte"]), **sizes, redis_client=env, subscriber=env, socket=env, poller=env,
        clock=env.clock), pipelines)


class _ReferencePushDispatcher:
    """Stand-in for task_dispatcher.PushDispatcher (:188-419), which imports zmq and
    redis at module level: the reference's method names, each failing if the
    subclass ever reaches it, plus one method only the base defines."""

    def __init__(self, *args, **kwargs):
        raise AssertionError("the reference __init__ must not run")

    def _unreachable(self, *args, **kwargs):
        raise AssertionError("a reference method was reached")

    bind_socket = send_message = receive_message = query_redis = _unreachable
    purge_workers = start = start_heartbeat = _unreachable

    def base_only(self):
        return "inherited"


def test_subclass_of_the_reference_class(dispatcher_cls):
    """GpuPushDispatcher.subclass_of(PushDispatcher): an instance of the
    reference's class whose reference methods are all the GPU ones; the golden
    replays pass through it unchanged."""
    Sub = dispatcher_cls.subclass_of(_ReferencePushDispatcher)
    for path in (GOLDEN[0], GOLDEN[-1]):
        z = np.load(path)
        d = replay_golden(z, lambda sizes, env: Sub(
            "127.0.0.1", 0, float(z["tte"]), **sizes, redis_client=env, subscriber=env, socket=env, poller=env,
            clock=env.clock))
        assert isinstance(d, _ReferencePushDispatcher) and isinstance(d, dispatcher_cls)
        assert d.base_only() == "inherited"
        assert isinstance(d.purge_workers(), list)  # the GPU purge, not the base's


def golden_sizes(z):
    """Table sizes for replaying golden vector z through a dispatcher."""
    W = int(z["W"])
    max_e = max(1, int(np.diff(z["ev_off"]).max(initial=0)))
    return dict(max_workers=2 * W + max_e, max_events=max_e + 1,
                max_inflight=len(z["init_log"]) + len(z["exp_assign"]) + 64)


def replay_golden(z, make_dispatcher, pipelines=True):
    """Replay a reference-captured golden vector (tests/golden/*.npz) through the
    dispatcher make_dispatcher(sizes, env) builds, checking every message, Redis
    write, pending task, LRU queue entry and worker record per tick."""
    W = int(z["W"])
    T = int(z["n_ticks"])
    env = FakeEnv(pipelines)
    d = make_dispatcher(golden_sizes(z), env)
    reg0 = z["init_reg"].astype(bool)
    # test-side model of the in-flight records (golden sequence numbering)
    seq_tid, seq_slot, inflight = {}, {}, set()
    for q, s in enumerate(z["init_log"]):
        seq_tid[q] = "init%d" % q
        seq_slot[q] = int(s)
        if s >= 0 and reg0[s] and z["init_epoch"][s] == 0:
            inflight.add(q)
    d.restore(dict(reg=z["init_reg"], free=z["init_free"], hb=z["init_hb"], epoch=z["init_epoch"],
                   queue=z["init_queue"], log=z["init_log"],
                   identity=[wid(s) if reg0[s] else None for s in range(W)],
                   inflight={q: (seq_tid[q], seq_slot[q]) for q in inflight}))
    head = len(z["init_log"])
    carried = []
    for t in range(T):
        e0, e1 = int(z["ev_off"][t]), int(z["ev_off"][t + 1])
        rec = z["exp_reconnect"][e0:e1]
        exp_sent, exp_hset = [], []
        for i in range(e0, e1):
            k, s, v, ts = int(z["ev_kind"][i]), int(z["ev_slot"][i]), int(z["ev_val"][i]), float(z["ev_ts"][i])
            m = {"type": KIND_MSG[k]}
            if k == 0:
                m["data"] = {"num_processes": v}
            elif k == 1:
                m["data"] = {"free_processes": v}
            elif k == 3:
                q = int(z["ev_seq"][i])
                live = q >= 0 and q in inflight and seq_slot[q] == s
                tid = seq_tid[q] if live else "stale-%d-%d" % (t, i)
                m["data"] = {"task_id": tid, "status": "COMPLETED", "result": "r%d" % i}
                if not rec[i - e0]:
                    exp_hset.append((tid, {"status": "COMPLETED", "result": "r%d" % i}))
                    if live:
                        inflight.discard(q)
            env.inbound.append((wid(s), codec.serialize(m).encode("utf-8"), ts))
            if rec[i - e0]:
                exp_sent.append((wid(s), {"type": "reconnect"}))
        new = ["t%d_%d" % (t, j) for j in range(int(z["n_new"][t]))]
        env.tasks.extend(new)
        env.now = float(z["now"][t])
        a0, a1 = int(z["exp_assign_off"][t]), int(z["exp_assign_off"][t + 1])
        o0, o1 = int(z["exp_orphan_off"][t]), int(z["exp_orphan_off"][t + 1])
        orph = [int(q) for q in z["exp_orphan"][o0:o1]]
        for q in orph:
            inflight.discard(q)
        pending = [seq_tid[q] for q in orph] + carried + new
        assign = z["exp_assign"][a0:a1]
        for k, s in enumerate(assign):
            tid = pending[k]
            exp_sent.append((wid(s), {"type": "task", "data": {"task_id": tid, "fn_payload": "fn_payload:" + tid,
                                                               "param_payload": "param_payload:" + tid}}))
            exp_hset.append((tid, {"status": "RUNNING"}))
            seq_tid[head + k] = tid
            seq_slot[head + k] = int(s)
            inflight.add(head + k)
        head += len(assign)
        carried = pending[len(assign):]
        env.sent.clear()
        env.hsets.clear()
        d.tick()
        assert env.sent == exp_sent, "tick %d: sent messages differ" % t
        assert env.hsets == exp_hset, "tick %d: redis writes differ" % t
        assert list(d.pending) == carried, "tick %d: pending tasks differ" % t
        q0, q1 = int(z["exp_post_queue_off"][t]), int(z["exp_post_queue_off"][t + 1])
        assert d.free_workers == [wid(s) for s in z["exp_post_queue"][q0:q1]], "tick %d: LRU queue" % t
        workers = d.workers
        exp_reg = np.nonzero(z["exp_post_reg"][t])[0]
        assert sorted(workers) == sorted(wid(s) for s in exp_reg), "tick %d: registered workers" % t
        for s in exp_reg:
            w = workers[wid(s)]
            assert w.free_processes == int(z["exp_post_free"][t][s]), "tick %d slot %d free" % (t, s)
            assert w.last_heartbeat == float(z["exp_post_hb"][t][s]), "tick %d slot %d hb" % (t, s)
    return d


def test_dispatcher_log_compaction_keeps_results(dispatcher_cls):
    """A tiny in-flight log forces compact_log() every few ticks; assignments must
    still equal a run with a large log."""
    GpuPushDispatcher = dispatcher_cls

    runs = []
    for cap in (1 << 16, 40):
        env = FakeEnv()
        d = GpuPushDispatcher("127.0.0.1", 0, 10, max_workers=16, max_events=64, max_inflight=cap,
                              redis_client=env, subscriber=env, socket=env, poller=env, clock=env.clock)
        sent = []
        for t in range(16):
            env.now = 1000.0 + t
            if t == 0:
                for w in range(6):
                    env.inbound.append((wid(w), codec.serialize(
                        {"type": "register", "data": {"num_processes": 3}}).encode(), env.now))
            else:
                # every worker returns one result per tick, worker 5 goes silent after tick 3
                for (dst, m) in list(prev):
                    if m["type"] == "task" and not (dst == wid(5) and t > 3):
                        env.inbound.append((dst, codec.serialize({"type": "result", "data": {
                            "task_id": m["data"]["task_id"], "status": "COMPLETED", "result": 1}}).encode(),
                            env.now))
                env.now += 0.5
            env.tasks.extend("t%d_%d" % (t, j) for j in range(7))
            env.sent.clear()
            d.tick()
            prev = list(env.sent)
            sent.append(prev)
        runs.append(sent)
        assert (d.compactions > 0) == (cap == 40)
    assert runs[0] == runs[1]
    assert sum(len(x) for x in runs[0]) > 50


def test_backlog_beyond_log_compacts_rarely(dispatcher_cls):
    """A task backlog far larger than the in-flight log: dispatches are bounded by
    the workers' free capacity (4 per tick here), so the log is compacted only when
    that reclaims a quarter of it -- not on every tick -- and the dispatches equal a
    run with a log large enough never to compact."""
    runs, comp = [], []
    for cap in (1 << 16, 64):
        env = FakeEnv()
        d = dispatcher_cls("127.0.0.1", 0, 10, max_workers=8, max_events=64, max_inflight=cap,
                           redis_client=env, subscriber=env, socket=env, poller=env, clock=env.clock)
        env.tasks.extend("b%d" % j for j in range(400))
        sent, prev = [], []
        for t in range(40):
            env.now = 1000.0 + t
            if t == 0:
                for w in range(2):
                    env.inbound.append((wid(w), codec.serialize(
                        {"type": "register", "data": {"num_processes": 2}}).encode(), env.now))
            for (dst, m) in prev:
                if m["type"] == "task":
                    env.inbound.append((dst, codec.serialize({"type": "result", "data": {
                        "task_id": m["data"]["task_id"], "status": "COMPLETED", "result": 1}}).encode(), env.now))
            env.sent.clear()
            d.tick()
            prev = list(env.sent)
            sent.append(prev)
        runs.append(sent)
        comp.append(d.compactions)
    assert runs[0] == runs[1]
    assert sum(len(x) for x in runs[0]) >= 4 * 39
    assert comp[0] == 0 and 0 < comp[1] <= 40 // 3, comp


def test_enospc_rerun_renumbers_result_sequences(dispatcher_cls):
    """A tick that carries results and whose dispatches overflow the in-flight log
    (the pre-check does not compact: too little garbage) fails with FB_ENOSPC; the
    dispatcher compacts -- renumbering every in-flight sequence -- and reruns the
    tick with the results' sequence numbers looked up again.  Afterwards the
    finished tasks must not be redistributed when their workers die: every sent
    message equals a run whose log never fills (dispatcher.py ENOSPC)."""
    runs, comp = [], []
    for cap in (1 << 16, 64):
        env = FakeEnv()
        d = dispatcher_cls("127.0.0.1", 0, 10, max_workers=8, max_events=128, max_inflight=cap,
                           redis_client=env, subscriber=env, socket=env, poller=env, clock=env.clock)
        env.tasks.extend("e%d" % j for j in range(65))
        sent, prev = [], []
        for t in range(6):
            env.now = 1000.0 + t
            if t == 0:  # two workers with one process each: 2 dispatches per tick
                for w in range(2):
                    env.inbound.append((wid(w), codec.serialize(
                        {"type": "register", "data": {"num_processes": 1}}).encode(), env.now))
            if t == 2:  # a large worker: this tick dispatches 61 tasks (head 4 + 61 > 64)
                env.inbound.append((wid(2), codec.serialize(
                    {"type": "register", "data": {"num_processes": 59}}).encode(), env.now))
            for (dst, m) in prev:
                # every result comes back through tick 2; at tick 3 only worker 2's,
                # then every worker falls silent
                if m["type"] == "task" and (t <= 2 or (t == 3 and dst == wid(2))):
                    env.inbound.append((dst, codec.serialize({"type": "result", "data": {
                        "task_id": m["data"]["task_id"], "status": "COMPLETED", "result": 1}}).encode(), env.now))
            if t == 5:
                env.now = 1000.0 + 20  # every heartbeat expired: the unfinished tasks are orphans
                env.inbound.append((wid(3), codec.serialize(
                    {"type": "register", "data": {"num_processes": 10}}).encode(), env.now))
            env.sent.clear()
            d.tick()
            prev = list(env.sent)
            sent.append(prev)
        runs.append(sent)
        comp.append(d.compactions)
    assert comp[0] == 0 and comp[1] >= 2, comp
    assert runs[0] == runs[1]
    # the last tick redistributes exactly the two unfinished tasks of workers 0 and 1
    redistributed = [m["data"]["task_id"] for _, m in runs[1][5] if m["type"] == "task"]
    unfinished = [m["data"]["task_id"] for dst, m in runs[1][2] if m["type"] == "task" and dst != wid(2)]
    assert sorted(redistributed) == sorted(unfinished) and len(unfinished) == 2


def test_purge_workers_evicts_without_dispatching(dispatcher_cls):
    """purge_workers() (task_dispatcher.py:241-249) deletes the expired records and
    sends nothing; the dead worker's in-flight tasks go to the front of the pending
    tasks and the next tick dispatches them first (the reference loses them)."""
    GpuPushDispatcher = dispatcher_cls
    env = FakeEnv()
    d = GpuPushDispatcher("127.0.0.1", 0, 10, max_workers=16, max_events=64, max_inflight=1 << 12,
                          redis_client=env, subscriber=env, socket=env, poller=env, clock=env.clock)
    env.now = 1000.0
    for w in range(4):
        env.inbound.append((wid(w), codec.serialize({"type": "register", "data": {"num_processes": 2}}).encode(),
                            1000.0))
    env.tasks.extend("t%d" % j for j in range(6))
    d.tick()
    first = [(dst, m["data"]["task_id"]) for dst, m in env.sent if m["type"] == "task"]
    assert len(first) == 6
    # workers 1..3 keep sending heartbeats; worker 0 goes silent and expires
    env.now = 1005.0
    for w in (1, 2, 3):
        env.inbound.append((wid(w), codec.serialize({"type": "heartbeat"}).encode(), 1005.0))
    d.tick()
    env.sent.clear()
    env.hsets.clear()
    env.t = 1010.5  # worker 0's last heartbeat is 10.5 s old, the others' 5.5 s
    gone = d.purge_workers()
    assert gone == [wid(0)]
    assert env.sent == [] and env.hsets == []  # purge sends and writes nothing
    lost = [tid for dst, tid in first if dst == wid(0)]
    assert lost and list(d.pending)[:len(lost)] == lost
    assert wid(0) not in d.workers and wid(0) not in d.free_workers
    env.now = 1011.0
    d.tick()
    redone = [m["data"]["task_id"] for dst, m in env.sent if m["type"] == "task"]
    assert redone[:len(lost)] == lost and all(dst != wid(0) for dst, _ in env.sent)


DEQUE = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "deque_*.npz")))


@pytest.mark.parametrize("path", DEQUE, ids=[os.path.basename(p)[:-4] for p in DEQUE])
def test_dispatcher_start_replays_reference(path, dispatcher_cls, pipelines):
    """``start()`` (the loop without heartbeats, task_dispatcher.py:251-322) on the
    vectors captured from the reference's start(): task messages, Redis writes,
    the deque (identities repeated) and the worker records."""
    z = np.load(path)
    W = int(z["W"])
    max_e = max(1, int(np.diff(z["ev_off"]).max(initial=0)))
    env = FakeEnv(pipelines)
    d = dispatcher_cls("127.0.0.1", 0, 10, max_workers=2 * W + max_e, max_events=max_e + 1,
                       max_inflight=len(z["init_log"]) + len(z["exp_assign"]) + 64,
                       redis_client=env, subscriber=env, socket=env, poller=env, clock=env.clock)
    d.use_loop("deque")
    reg0 = z["init_reg"].astype(bool)
    seq_tid, seq_slot, inflight = {}, {}, set()
    for q, s in enumerate(z["init_log"]):
        seq_tid[q], seq_slot[q] = "init%d" % q, int(s)
        if s >= 0:
            inflight.add(q)
    d.restore(dict(reg=z["init_reg"], free=z["init_free"], hb=z["init_hb"], epoch=z["init_epoch"],
                   queue=z["init_queue"], log=z["init_log"],
                   identity=[wid(s) if reg0[s] else None for s in range(W)],
                   inflight={q: (seq_tid[q], seq_slot[q]) for q in inflight}))
    head = len(z["init_log"])
    carried = []
    for t in range(int(z["n_ticks"])):
        e0, e1 = int(z["ev_off"][t]), int(z["ev_off"][t + 1])
        exp_sent, exp_hset = [], []
        for i in range(e0, e1):
            k, s, v, ts = int(z["ev_kind"][i]), int(z["ev_slot"][i]), int(z["ev_val"][i]), float(z["ev_ts"][i])
            m = {"type": KIND_MSG[k]}
            if k == 0:
                m["data"] = {"num_processes": v}
            elif k == 1:
                m["data"] = {"free_processes": v}
            elif k == 3:
                q = int(z["ev_seq"][i])
                live = q >= 0 and q in inflight and seq_slot[q] == s
                tid = seq_tid[q] if live else "stale-%d-%d" % (t, i)
                m["data"] = {"task_id": tid, "status": "COMPLETED", "result": "r%d" % i}
                exp_hset.append((tid, {"status": "COMPLETED", "result": "r%d" % i}))
                if live:
                    inflight.discard(q)
            env.inbound.append((wid(s), codec.serialize(m).encode("utf-8"), ts))
        new = ["t%d_%d" % (t, j) for j in range(int(z["n_new"][t]))]
        env.tasks.extend(new)
        env.now = float(z["now"][t])
        a0, a1 = int(z["exp_assign_off"][t]), int(z["exp_assign_off"][t + 1])
        pending = carried + new
        assign = z["exp_assign"][a0:a1]
        for k, s in enumerate(assign):
            tid = pending[k]
            exp_sent.append((wid(s), {"type": "task", "data": {"task_id": tid, "fn_payload": "fn_payload:" + tid,
                                                               "param_payload": "param_payload:" + tid}}))
            exp_hset.append((tid, {"status": "RUNNING"}))
            seq_tid[head + k], seq_slot[head + k] = tid, int(s)
            inflight.add(head + k)
        head += len(assign)
        carried = pending[len(assign):]
        env.sent.clear()
        env.hsets.clear()
        d.tick()
        assert env.sent == exp_sent, "tick %d: sent messages differ" % t
        assert env.hsets == exp_hset, "tick %d: redis writes differ" % t
        assert list(d.pending) == carried, "tick %d: pending tasks differ" % t
        q0, q1 = int(z["exp_post_queue_off"][t]), int(z["exp_post_queue_off"][t + 1])
        assert d.free_workers == [wid(s) for s in z["exp_post_queue"][q0:q1]], "tick %d: deque" % t
        workers = d.workers
        exp_reg = np.nonzero(z["exp_post_reg"][t])[0]
        assert sorted(workers) == sorted(wid(s) for s in exp_reg), "tick %d: registered workers" % t
        for s in exp_reg:
            assert workers[wid(s)].free_processes == int(z["exp_post_free"][t][s]), "tick %d slot %d" % (t, s)


def test_dispatcher_start_unknown_result_does_not_kill_the_loop(dispatcher_cls):
    """The reference's start() HSETs a result from an unknown identity and then
    raises KeyError (:288-291); the drop-in keeps the HSET and drops the message."""
    env = FakeEnv()
    d = dispatcher_cls("127.0.0.1", 0, 10, max_workers=8, max_events=16, max_inflight=64,
                       redis_client=env, subscriber=env, socket=env, poller=env, clock=env.clock)
    d.use_loop("deque")
    env.inbound.append((b"ghost", codec.serialize({"type": "result", "data": {
        "task_id": "tX", "status": "COMPLETED", "result": 1}}).encode(), 0.0))
    env.inbound.append((b"w1", codec.serialize({"type": "register", "data": {"num_processes": 2}}).encode(), 0.0))
    env.tasks.extend(["a", "b", "c"])
    res = d.tick()
    assert res["unknown_results"] == 1
    assert env.hsets[0] == ("tX", {"status": "COMPLETED", "result": 1})
    assert [m["data"]["task_id"] for _, m in env.sent] == ["a", "b"]
    assert list(d.pending) == ["c"]
    assert b"ghost" not in d.workers


def test_batched_io_round_trips(dispatcher_cls):
    """Pipelined host I/O: 2 Redis round trips for a tick's dispatches (+1 for its
    results) instead of 3 per task (+1 per result); same messages and writes."""
    runs = []
    for pipelines in (True, False):
        env = FakeEnv(pipelines)
        d = dispatcher_cls("127.0.0.1", 0, 10, max_workers=16, max_events=64, max_inflight=4096,
                           redis_client=env, subscriber=env, socket=env, poller=env, clock=env.clock)
        for w in range(4):
            env.inbound.append((wid(w), codec.serialize({"type": "register", "data": {"num_processes": 8}}).encode(),
                                0.0))
        env.tasks.extend("t%d" % j for j in range(20))
        env.now = 1.0
        d.tick()
        trips0 = env.round_trips
        env.inbound.append((wid(0), codec.serialize({"type": "result", "data": {
            "task_id": "t0", "status": "COMPLETED", "result": 1}}).encode(), 1.5))
        env.tasks.extend("u%d" % j for j in range(5))
        env.now = 2.0
        d.tick()
        runs.append((env.sent, env.hsets, trips0, env.round_trips - trips0))
    (s1, h1, a1, b1), (s2, h2, a2, b2) = runs
    assert s1 == s2 and h1 == h2
    assert (a1, b1) == (2, 3) and (a2, b2) == (3 * 20, 1 + 3 * 5)


def _dill_wire(obj):
    import codecs as _c
    import dill
    return _c.encode(dill.dumps(obj), "base64").decode()  # helper_functions.py:5-6


def test_codec_bytes_equal_dill_for_messages():
    """The C-pickler path writes exactly dill's bytes for every message shape the
    dispatcher and workers exchange."""
    msgs = [{"type": "task", "data": {"task_id": "0f8fad5b-d9cb-469f-a165-70867728950e",
                                      "fn_payload": "gASV" * 60, "param_payload": "gAS" * 30}},
            {"type": "reconnect"}, {"type": "wait"}, {"type": "heartbeat"},
            {"type": "register", "data": {"num_processes": 8}},
            {"type": "reconnect", "data": {"free_processes": -1}},
            {"type": "result", "data": {"task_id": "t1", "status": "COMPLETED", "result": "gASVBQ=="}},
            {"type": "result", "data": {"task_id": "t1", "status": "FAILED", "result": None}}]
    for m in msgs:
        assert codec.serialize(m) == _dill_wire(m), m
        assert codec.deserialize(codec.serialize(m)) == m


def test_codec_random_plain_data_matches_dill():
    hypothesis = pytest.importorskip("hypothesis")
    st = hypothesis.strategies
    leaves = st.one_of(st.none(), st.booleans(), st.integers(-2 ** 70, 2 ** 70),
                       st.floats(allow_nan=False), st.text(max_size=40), st.binary(max_size=40))
    data = st.recursive(leaves, lambda ch: st.one_of(st.lists(ch, max_size=5), st.tuples(ch, ch),
                                                     st.dictionaries(st.text(max_size=8), ch, max_size=5)),
                        max_leaves=20)

    @hypothesis.settings(max_examples=300, deadline=None)
    @hypothesis.given(data)
    def check(obj):
        assert codec.serialize(obj) == _dill_wire(obj)

    check()


def test_codec_non_plain_objects_go_through_dill():
    import dill

    def double(x):
        return 2 * x
    s = codec.serialize(double)
    assert codec.deserialize(s)(21) == 42
    assert dill.loads(__import__("codecs").decode(s.encode(), "base64"))(4) == 8
