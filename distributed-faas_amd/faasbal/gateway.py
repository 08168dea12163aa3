"""REST gateway of the service.

The reference repository ships the dispatchers and workers but not the REST
front end its clients talk to.  Its shape is fixed by those clients:

* ``POST /register_function`` ``{"name", "payload"}`` -> ``{"function_id"}``
  (client_performance.py:101-104, test_suit.py:39-43)
* ``POST /execute_function`` ``{"function_id", "payload"}`` -> ``{"task_id"}``
  (client_performance.py:111-116, test_suit.py:45-53)
* ``GET /status/{task_id}`` -> ``{"task_id", "status"}`` with status in
  QUEUED / RUNNING / COMPLETED / FAILED (test_suit.py:19, :55-59)
* ``GET /result/{task_id}`` -> ``{"task_id", "status", "result"}``
  (client_performance.py:121-124, test_suit.py:80-92)

and the task record it must leave for the dispatchers by the reference's
own producer (old/client_debug.py:40-47, task_dispatcher.py:38-52):
``HSET <task_id> status=QUEUED fn_payload=... param_payload=... result=None``
then ``PUBLISH tasks <task_id>`` on the channel of config.ini:8.  Payloads are
the clients' dill+base64 strings, stored and forwarded untouched.

``MemoryRedis`` is an in-process stand-in for the redis-py client (hashes,
pub/sub, non-transactional pipelines) for tests and single-host runs: no Redis
server exists in this image.  With a real ``redis.Redis`` every request is
one round trip, ``execute_function`` two (HGET of the function, then record +
publish pipelined).
"""

import collections
import threading
import uuid

VALID_STATUSES = ("QUEUED", "RUNNING", "COMPLETED", "FAILED")


def _b(v):
    if isinstance(v, bytes):
        return v
    if isinstance(v, (bytearray, memoryview)):
        return bytes(v)
    return str(v).encode("utf-8")


def _s(v):
    return v.decode("utf-8") if isinstance(v, (bytes, bytearray)) else v


class _PubSub:
    """redis-py ``PubSub`` subset: subscribe + non-blocking get_message."""

    def __init__(self, store):
        self._store = store
        self._q = collections.deque()
        self.channels = set()

    def subscribe(self, *channels):
        with self._store._lock:
            for ch in channels:
                ch = _s(ch)
                self.channels.add(ch)
                self._store._subs[ch].append(self)
                self._q.append({"type": "subscribe", "pattern": None, "channel": _b(ch),
                                "data": len(self.channels)})

    def get_message(self, ignore_subscribe_messages=False, timeout=0.0):
        with self._store._lock:
            while self._q:
                m = self._q.popleft()
                if ignore_subscribe_messages and m["type"] != "message":
                    continue
                return m
        return None


class _Pipeline:
    """Non-transactional pipeline: commands queue up and run in order on execute()."""

    def __init__(self, store):
        self._store, self._cmds = store, []

    def __getattr__(self, name):
        fn = getattr(self._store, name)

        def queue(*a, **k):
            self._cmds.append((fn, a, k))
            return self
        return queue

    def execute(self):
        with self._store._lock:
            self._store.round_trips += 1
            out = [fn(*a, _rt=False, **k) for fn, a, k in self._cmds]
        self._cmds = []
        return out

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self._cmds = []


class MemoryRedis:
    """Thread-safe in-memory redis-py stand-in (hset/hget/hgetall/exists/publish/
    pubsub/pipeline); values come back as bytes like redis-py's default client.
    ``round_trips`` counts client round trips (one per command, one per pipeline)."""

    def __init__(self):
        self._lock = threading.RLock()
        self._h = {}
        self._subs = collections.defaultdict(list)
        self.round_trips = 0

    def _rt(self, rt):
        if rt:
            self.round_trips += 1

    def hset(self, name, key=None, value=None, mapping=None, _rt=True):
        with self._lock:
            self._rt(_rt)
            h = self._h.setdefault(_b(name), {})
            items = dict(mapping or {})
            if key is not None:
                items[key] = value
            n = 0
            for k, v in items.items():
                n += _b(k) not in h
                h[_b(k)] = _b(v)
            return n

    def hget(self, name, key, _rt=True):
        with self._lock:
            self._rt(_rt)
            return self._h.get(_b(name), {}).get(_b(key))

    def hgetall(self, name, _rt=True):
        with self._lock:
            self._rt(_rt)
            return dict(self._h.get(_b(name), {}))

    def exists(self, *names, _rt=True):
        with self._lock:
            self._rt(_rt)
            return sum(_b(n) in self._h for n in names)

    def publish(self, channel, message, _rt=True):
        with self._lock:
            self._rt(_rt)
            subs = self._subs.get(_s(channel), [])
            for s in subs:
                s._q.append({"type": "message", "pattern": None, "channel": _b(channel), "data": _b(message)})
            return len(subs)

    def pubsub(self):
        return _PubSub(self)

    def pipeline(self, transaction=True):
        return _Pipeline(self)


class Gateway:
    """The service's REST operations over a redis-py style client, framework-free
    (``create_app`` mounts them on FastAPI)."""

    def __init__(self, redis_client=None, tasks_channel="tasks"):
        if redis_client is None:
            import redis  # the reference's store (config.ini:6-9); only when none is injected
            redis_client = redis.Redis(host="localhost", port=6379, db=1)
        self.r = redis_client
        self.channel = tasks_channel

    def _pipe(self):
        mk = getattr(self.r, "pipeline", None)
        return mk(transaction=False) if mk is not None else None

    def register_function(self, name: str, payload: str) -> dict:
        fid = str(uuid.uuid4())
        self.r.hset(fid, mapping={"name": name, "payload": payload})
        return {"function_id": fid}

    def execute_function(self, function_id: str, payload: str):
        """-> {"task_id"}, or None when the function id is unknown."""
        fn = self.r.hget(function_id, "payload")
        if fn is None:
            return None
        tid = str(uuid.uuid4())
        rec = {"status": "QUEUED", "fn_payload": fn, "param_payload": payload, "result": "None"}
        p = self._pipe()
        if p is not None:
            p.hset(tid, mapping=rec)
            p.publish(self.channel, tid)
            p.execute()
        else:
            self.r.hset(tid, mapping=rec)
            self.r.publish(self.channel, tid)
        return {"task_id": tid}

    def status(self, task_id: str):
        st = self.r.hget(task_id, "status")
        return None if st is None else {"task_id": task_id, "status": _s(st)}

    def result(self, task_id: str):
        h = self.r.hgetall(task_id)
        if not h or b"status" not in h:
            return None
        return {"task_id": task_id, "status": _s(h[b"status"]), "result": _s(h.get(b"result", b"None"))}


def create_app(redis_client=None, tasks_channel="tasks"):
    """FastAPI app with the four endpoints the reference's clients call."""
    from fastapi import FastAPI, HTTPException
    from pydantic import BaseModel

    class RegisterFn(BaseModel):
        name: str
        payload: str

    class ExecuteFn(BaseModel):
        function_id: str
        payload: str

    gw = Gateway(redis_client, tasks_channel)
    app = FastAPI(title="Distributed-FaaS gateway")
    app.state.gateway = gw

    @app.post("/register_function")
    def register_function(body: RegisterFn):
        return gw.register_function(body.name, body.payload)

    @app.post("/execute_function")
    def execute_function(body: ExecuteFn):
        out = gw.execute_function(body.function_id, body.payload)
        if out is None:
            raise HTTPException(status_code=404, detail="unknown function_id %s" % body.function_id)
        return out

    @app.get("/status/{task_id}")
    def status(task_id: str):
        out = gw.status(task_id)
        if out is None:
            raise HTTPException(status_code=404, detail="unknown task_id %s" % task_id)
        return out

    @app.get("/result/{task_id}")
    def result(task_id: str):
        out = gw.result(task_id)
        if out is None:
            raise HTTPException(status_code=404, detail="unknown task_id %s" % task_id)
        return out

    return app


def main(argv=None):
    """``python -m faasbal.gateway [--host 127.0.0.1 --port 8000]`` against
    localhost Redis db 1 (the reference clients' base_url, test_suit.py:17)."""
    import argparse

    import uvicorn
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--memory", action="store_true", help="in-process MemoryRedis instead of localhost Redis")
    a = ap.parse_args(argv)
    uvicorn.run(create_app(MemoryRedis() if a.memory else None), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
