"""REST gateway (faasbal.gateway).

The reference holds no gateway; its clients fix the API.  These tests replay
the reference's own client tests (test_suit.py:38-92) against the FastAPI app
in-process, check the Redis task record against the reference producer
(old/client_debug.py:40-47) and run the whole service in one process:
client -> gateway -> Redis pub/sub -> GpuPushDispatcher -> push workers
(push_worker.py:45-97 semantics, helper_functions.py:11-28) -> Redis -> client.
"""
import collections
import random

import pytest

from faasbal import codec
from faasbal.gateway import VALID_STATUSES, Gateway, MemoryRedis, create_app

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402


def double(x):
    return x * 2


def boom(x):
    raise ValueError(x)


@pytest.fixture
def svc():
    r = MemoryRedis()
    sub = r.pubsub()
    sub.subscribe("tasks")
    return r, sub, TestClient(create_app(r))


def test_execute_fn(svc):
    """test_suit.py:38-59."""
    r, sub, c = svc
    resp = c.post("/register_function", json={"name": "hello", "payload": codec.serialize(double)})
    assert resp.status_code == 200 and "function_id" in resp.json()
    fid = resp.json()["function_id"]
    resp = c.post("/execute_function", json={"function_id": fid, "payload": codec.serialize(((2,), {}))})
    assert resp.status_code == 200 and "task_id" in resp.json()
    tid = resp.json()["task_id"]
    resp = c.get("/status/%s" % tid)
    assert resp.status_code == 200
    assert resp.json() == {"task_id": tid, "status": "QUEUED"}
    assert resp.json()["status"] in VALID_STATUSES


def test_task_record_matches_reference_producer(svc):
    """HSET task_id {status, fn_payload, param_payload, result} + PUBLISH tasks task_id
    (old/client_debug.py:40-47) -- what TaskDispatcher.query_redis reads (:38-52)."""
    r, sub, c = svc
    fn, par = codec.serialize(double), codec.serialize(((5,), {}))
    fid = c.post("/register_function", json={"name": "double", "payload": fn}).json()["function_id"]
    tid = c.post("/execute_function", json={"function_id": fid, "payload": par}).json()["task_id"]
    assert r.hgetall(tid) == {b"status": b"QUEUED", b"fn_payload": fn.encode(), b"param_payload": par.encode(),
                              b"result": b"None"}
    m = sub.get_message()
    assert m["type"] == "subscribe"
    m = sub.get_message()
    assert m["type"] == "message" and m["channel"] == b"tasks" and m["data"] == tid.encode()
    assert sub.get_message() is None
    # the payloads run as the worker would run them (helper_functions.py:11-28)
    assert codec.deserialize(r.hget(tid, "fn_payload").decode())(*codec.deserialize(par)[0]) == 10


def test_roundtrip(svc):
    """test_suit.py:62-92: a worker completes the task, the client reads the result."""
    r, sub, c = svc
    fid = c.post("/register_function", json={"name": "double", "payload": codec.serialize(double)}).json()
    number = random.Random(3).randint(0, 10000)
    tid = c.post("/execute_function", json={"function_id": fid["function_id"],
                                            "payload": codec.serialize(((number,), {}))}).json()["task_id"]
    r.hset(tid, mapping={"status": "RUNNING"})
    assert c.get("/result/%s" % tid).json()["status"] == "RUNNING"
    r.hset(tid, mapping={"status": "COMPLETED", "result": codec.serialize(number * 2)})
    s = c.get("/result/%s" % tid).json()
    assert s["task_id"] == tid and s["status"] == "COMPLETED"
    assert codec.deserialize(s["result"]) == number * 2


def test_unknown_ids_are_404(svc):
    r, sub, c = svc
    assert c.post("/execute_function", json={"function_id": "nope", "payload": "x"}).status_code == 404
    assert c.get("/status/nope").status_code == 404
    assert c.get("/result/nope").status_code == 404
    assert c.post("/register_function", json={"name": "x"}).status_code == 422  # payload missing


def test_execute_is_two_round_trips():
    """One HGET of the function, then record + publish in one pipeline."""
    r = MemoryRedis()
    g = Gateway(r)
    fid = g.register_function("f", "p")["function_id"]
    n0 = r.round_trips
    g.execute_function(fid, "q")
    assert r.round_trips - n0 == 2


class _NoPipe:
    """Client without pipeline(): the gateway falls back to one command per call."""

    def __init__(self, r):
        self.r = r

    def __getattr__(self, k):
        if k == "pipeline":
            raise AttributeError(k)
        return getattr(self.r, k)


def test_execute_without_pipelines_same_record():
    r = MemoryRedis()
    sub = r.pubsub()
    sub.subscribe("tasks")
    g = Gateway(_NoPipe(r))
    fid = g.register_function("f", "p")["function_id"]
    tid = g.execute_function(fid, "q")["task_id"]
    assert r.hgetall(tid) == {b"status": b"QUEUED", b"fn_payload": b"p", b"param_payload": b"q", b"result": b"None"}
    sub.get_message()
    assert sub.get_message()["data"] == tid.encode()


# ------------------------------------------------------------------ end to end

class _Router:
    """In-memory ROUTER socket + poller between the dispatcher and push workers."""

    def __init__(self):
        self.inbound = collections.deque()
        self.outbound = collections.defaultdict(collections.deque)

    def poll(self, timeout=None):
        return [(self, 1)] if self.inbound else []

    def recv_multipart(self):
        return list(self.inbound.popleft())

    def send_multipart(self, parts):
        self.outbound[parts[0]].append(parts[1])


class _PushWorker:
    """push_worker.PushWorker.start_heartbeat (push_worker.py:45-97), synchronous:
    register with n processes, run each task message (helper_functions.execute_fn)
    and answer with a result message."""

    def __init__(self, ident, n, router):
        self.id, self.n, self.router = ident, n, router

    def send(self, msg):
        self.router.inbound.append((self.id, codec.serialize(msg).encode("utf-8")))

    def register(self):
        self.send({"type": "register", "data": {"num_processes": self.n}})

    def step(self):
        q = self.router.outbound[self.id]
        while q:
            m = codec.deserialize(q.popleft().decode("utf-8"))
            if m["type"] == "reconnect":
                self.send({"type": "reconnect", "data": {"free_processes": self.n}})
                continue
            d = m["data"]
            fn = codec.deserialize(d["fn_payload"])
            args, kwargs = codec.deserialize(d["param_payload"])
            try:
                res, st = fn(*args, **kwargs), "COMPLETED"
            except Exception:
                res, st = None, "FAILED"
            self.send({"type": "result", "data": {"task_id": d["task_id"], "status": st,
                                                  "result": codec.serialize(res)}})


@pytest.fixture(params=[pytest.param("gpu", marks=pytest.mark.gpu), "host"])
def dispatcher_cls(request, monkeypatch):
    """Real balancer on the GPU; on the CPU the host logic over the oracle test
    double (tests/oracle_balancer.py)."""
    import faasbal.dispatcher as D
    if request.param == "host":
        from oracle_balancer import OracleBalancer
        monkeypatch.setattr(D, "GpuBalancer", OracleBalancer)
    return D.GpuPushDispatcher


def test_service_end_to_end(dispatcher_cls):
    """client_performance.measure_service (:98-130) in one process: 120 tasks
    (some failing) over 5 push workers, every result read back through REST."""
    r = MemoryRedis()
    router = _Router()
    clock = [100.0]
    d = dispatcher_cls("127.0.0.1", 0, 10, max_workers=64, max_inflight=4096, max_events=512,
                       redis_client=r, socket=router, poller=router, clock=lambda: clock[0])
    c = TestClient(create_app(r))
    workers = [_PushWorker(b"w%d" % i, 1 + i % 3, router) for i in range(5)]
    for w in workers:
        w.register()
    f_ok = c.post("/register_function", json={"name": "double", "payload": codec.serialize(double)}).json()
    f_bad = c.post("/register_function", json={"name": "boom", "payload": codec.serialize(boom)}).json()
    want = {}
    for i in range(120):
        fid = (f_bad if i % 17 == 5 else f_ok)["function_id"]
        tid = c.post("/execute_function", json={"function_id": fid,
                                                "payload": codec.serialize(((i,), {}))}).json()["task_id"]
        want[tid] = None if i % 17 == 5 else 2 * i
    for _ in range(400):
        clock[0] += 0.01
        d.tick()
        for w in workers:
            w.step()
        done = [c.get("/status/%s" % t).json()["status"] for t in want]
        if all(s in ("COMPLETED", "FAILED") for s in done):
            break
    for tid, v in want.items():
        s = c.get("/result/%s" % tid).json()
        assert s["status"] == ("FAILED" if v is None else "COMPLETED"), s
        assert codec.deserialize(s["result"]) == v
    assert not d.pending


def immediate_function(number):
    """client_performance.py:19-20, the no-op task of BASELINE configs[0]."""
    return number


@pytest.mark.parametrize("loop", ["heartbeat", "deque"])
def test_configs0_client_performance_shape(dispatcher_cls, loop):
    """BASELINE configs[0] as client_performance.py states it (:157-164, :218, :225-226):
    4 push workers of 4 processes each (``-w 4``, ``-np 4``), ``n_tasks`` 10 per worker ->
    a problem size of 40 ``immediate_function`` tasks with params ((1,), {})
    (``params_immediate_function``, :22-24); ``measure_service`` (:98-143) registers the
    function and the tasks over REST and polls every result until COMPLETED.  Both
    dispatcher loops: ``--hb`` (start_heartbeat) and the default ``start()``; every result
    is read back and checked."""
    r = MemoryRedis()
    router = _Router()
    clock = [100.0]
    d = dispatcher_cls("127.0.0.1", 0, 10, max_workers=64, max_inflight=4096, max_events=512,
                       redis_client=r, socket=router, poller=router, clock=lambda: clock[0])
    if loop == "deque":
        d.use_loop("deque")
    c = TestClient(create_app(r))
    number_workers, number_processes, n_tasks = 4, 4, 10
    workers = [_PushWorker(b"push%d" % i, number_processes, router) for i in range(number_workers)]
    for w in workers:
        w.register()
    fid = c.post("/register_function", json={"name": immediate_function.__name__,
                                              "payload": codec.serialize(immediate_function)}).json()["function_id"]
    problem_size = n_tasks * number_workers
    fn_params = [((1,), {}) for _ in range(problem_size)]
    tasks = [c.post("/execute_function", json={"function_id": fid, "payload": codec.serialize(p)}).json()["task_id"]
             for p in fn_params]
    assert len(set(tasks)) == problem_size
    for _ in range(200):
        clock[0] += 0.01
        d.tick()
        for w in workers:
            w.step()
        if all(c.get("/status/%s" % t).json()["status"] == "COMPLETED" for t in tasks):
            break
    for t, p in zip(tasks, fn_params):
        s = c.get("/result/%s" % t).json()
        assert s["status"] == "COMPLETED", s
        assert codec.deserialize(s["result"]) == immediate_function(*p[0], **p[1])
    assert not d.pending
    # every worker served: 40 tasks over 4 workers of 4 processes
    assert d.ticks > 1
