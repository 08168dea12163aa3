"""GpuPushDispatcher: drop-in for the reference's heartbeat ``PushDispatcher``.

Same constructor signature (``task_dispatcher.py:190``), same ZMQ ROUTER socket
and message flow, same Redis records and pub/sub channel, same wire codec.
What changes is the balancing state: the ``self.workers`` dict of
``PushWorker`` records (``:194, :203-212``), the ``free_workers`` LRU
OrderedDict (``:327``), ``purge_workers`` (``:241-249``) and the dispatch block
(``:393-419``) live on the GPU, in ``GpuBalancer`` (``libfaasbal.so`` through
ctypes).  The host loop works per *tick* instead of per message:

1. drain every inbound ZMQ message (``poll(0)`` until empty, ``:330-345``),
   stamping each with the clock at receipt, and map the worker identity
   (``bytes``) to a dense table slot;
2. drain every pending pub/sub task id (``get_message``, ``:394``);
3. one GPU tick: the messages' state updates (``:347-387``), the purge at
   ``now`` (``:390``), redistribution of dead workers' in-flight tasks
   (build-defined; the reference drops them, README.md:263-264) and the LRU
   dispatch of orphans then pending tasks;
4. the host I/O the reference does per message, in the same order: a
   ``reconnect`` request to unknown senders (``:356-358``), ``HSET`` of results
   from known workers (``:381``), then per dispatched task ``HGET`` x2
   (``query_redis``, ``:48-52``), ``send_message`` (``:410``) and
   ``HSET status=RUNNING`` (``:413``).

A tick is a legal arrival order for the reference loop (messages first, then
tasks): the assignments are bit-identical to the reference's on it
(tests/test_dispatcher.py replays the reference-captured goldens through this
class with fake sockets and Redis).

``start()`` runs the reference's loop without heartbeats
(``task_dispatcher.py:251-322``) the same way, on a deque-mode balancer: no
liveness, a ready deque that may repeat identities, results from an identity
without a record reported instead of crashing the loop (the reference raises
KeyError at ``:291``, after its ``HSET`` of the result).

There is no CPU path: the balancer is the HIP library, and constructing this
class without a GPU fails loudly.
"""
from __future__ import annotations

import collections
import time

import numpy as np

from . import codec
from ._lib import FB_ENOSPC, FB_EVS_RECONNECT, FaasbalError
from .balancer import GpuBalancer

EV_REGISTER, EV_RECONNECT, EV_HEARTBEAT, EV_RESULT, EV_OTHER = 0, 1, 2, 3, 4
_KINDS = {"register": EV_REGISTER, "reconnect": EV_RECONNECT, "heartbeat": EV_HEARTBEAT, "result": EV_RESULT}
_I32 = (-(1 << 31), (1 << 31) - 1)


class WorkerView:
    """Read-only stand-in for ``PushDispatcher.PushWorker`` (``:203-212``)."""

    __slots__ = ("free_processes", "last_heartbeat", "time_to_expire")

    def __init__(self, free_processes, last_heartbeat, time_to_expire):
        self.free_processes = int(free_processes)
        self.last_heartbeat = float(last_heartbeat)
        self.time_to_expire = time_to_expire

    def is_alive(self, now=None):
        now = time.time() if now is None else now
        return not (now - self.last_heartbeat > self.time_to_expire)


class GpuPushDispatcher:
    """Heartbeat push dispatcher whose balancing state lives on an MI355X.

    ``ip_address``, ``port``, ``time_to_expire``: as the reference
    (``task_dispatcher.py:190``; ``TIME_TO_EXPIRE`` of ``config.ini``).
    Keyword-only arguments size the device table and allow the transport objects
    to be injected (the defaults build exactly what the reference builds:
    ``redis.Redis(host='localhost', port=6379, db=1)`` subscribed to ``tasks``,
    and a bound ZMQ ROUTER with a ``zmq.Poller``).
    """

    def __init__(self, ip_address, port, time_to_expire=10, *, max_workers=65536, max_inflight=1 << 24,
                 max_events=65536, device=0, redis_client=None, subscriber=None, socket=None, poller=None,
                 clock=time.time, tasks_channel="tasks", batch_io=True, balancer=None):
        self.port = port
        self.batch_io = bool(batch_io)
        self.ip_address = ip_address
        self.time_to_expire = time_to_expire
        self.clock = clock
        # TaskDispatcher.__init__ (task_dispatcher.py:30-36)
        if redis_client is None:
            import redis  # the reference's client; only needed when none is injected
            redis_client = redis.Redis(host="localhost", port=6379, db=1)
        self.redis_client = redis_client
        if subscriber is None:
            subscriber = self.redis_client.pubsub()
            subscriber.subscribe(tasks_channel)
        self.subscriber = subscriber
        # PushDispatcher.__init__ (:196-201)
        if socket is None:
            self.bind_socket()
        else:
            self.socket = socket
        if poller is None:
            import zmq
            poller = zmq.Poller()
            poller.register(self.socket, zmq.POLLIN)
        self.poller = poller
        # device table: max_workers slots, all empty
        self.max_workers = int(max_workers)
        self.max_events = int(max_events)
        self.max_inflight = int(max_inflight)
        self.device = device
        self.mode = "heartbeat"
        # balancer: the worker table -- one GPU by default; a faasbal.sharded group for a
        # table sharded over several GPUs (same API, see ShardedPushDispatcher)
        self.balancer = balancer if balancer is not None else \
            GpuBalancer(self.max_workers, self.max_inflight, max_events=self.max_events, device=device)
        self._reset_host()
        W = self.max_workers
        self.balancer.load_state(np.zeros(W, np.uint8), np.zeros(W, np.int32), np.zeros(W, np.float64))
        self.ticks = 0
        self.compactions = 0

    @classmethod
    def subclass_of(cls, base):
        """This class as a subclass of the reference's ``PushDispatcher``
        (``task_dispatcher.py:188``), for code that type-checks or extends it:
        ``GpuPush = GpuPushDispatcher.subclass_of(PushDispatcher)``.  The methods
        here come first in the MRO, so every method the reference defines --
        ``bind_socket``, ``send_message``, ``receive_message``, ``query_redis``,
        ``purge_workers``, ``start``, ``start_heartbeat`` -- is the GPU one, and the
        reference's ``__init__`` (which binds a socket and opens Redis itself) is
        never run; anything else the base adds is inherited unchanged."""
        return type(cls.__name__, (cls, base), {"__doc__": cls.__doc__, "__module__": cls.__module__})

    def use_loop(self, mode):
        """Select the balancing loop before the first tick: ``"heartbeat"``
        (``start_heartbeat``, :324-419) or ``"deque"`` (``start``, :251-322).
        ``start()`` / ``start_heartbeat()`` call this themselves."""
        if mode == self.mode:
            return
        if self.ticks:
            raise FaasbalError(-6, "cannot switch the dispatcher loop after %d ticks" % self.ticks)
        if not isinstance(self.balancer, GpuBalancer):
            raise FaasbalError(-6, "the loop without heartbeats runs on a one-GPU balancer")
        self.balancer.close()
        self.balancer = GpuBalancer(self.max_workers, self.max_inflight, max_events=self.max_events,
                                    device=self.device, mode=mode)
        self.mode = mode
        W = self.max_workers
        self.balancer.load_state(np.zeros(W, np.uint8), np.zeros(W, np.int32), np.zeros(W, np.float64))

    def _reset_host(self):
        self.slot_of = {}                              # ZMQ identity -> slot
        self.identity = [None] * self.max_workers      # slot -> ZMQ identity
        self._free_slots = []                          # slots released by evictions (reused LIFO)
        self._next_slot = 0
        self.inflight = {}                             # log sequence -> (task_id, slot)
        self.task_seq = {}                             # task_id -> log sequence while in flight
        self.pending = collections.deque()             # task ids not yet dispatched (orphans first)
        self.head = 0                                  # in-flight log length
        self._last_ts = -np.inf

    # ------------------------------------------------ reference socket / Redis API
    def bind_socket(self):
        """Create and bind the ROUTER socket (``task_dispatcher.py:215-219``)."""
        import zmq
        self.socket = zmq.Context().socket(zmq.ROUTER)
        self.socket.bind(f"tcp://{self.ip_address}:{self.port}")

    def send_message(self, worker_id: bytes, message: object):
        """``:221-230``: dill+base64 payload to the worker identified by ``worker_id``."""
        self.socket.send_multipart([worker_id, codec.serialize(message).encode("utf-8")])

    def receive_message(self):
        """``:232-239``: (identity, deserialized message)."""
        worker, message = self.socket.recv_multipart()
        return worker, codec.deserialize(message.decode("utf-8"))

    def query_redis(self, message):
        """``TaskDispatcher.query_redis`` (``:38-52``)."""
        task_id = message["data"].decode("utf-8")
        fn_payload = self.redis_client.hget(task_id, "fn_payload")
        param_payload = self.redis_client.hget(task_id, "param_payload")
        return task_id, fn_payload.decode("utf-8"), param_payload.decode("utf-8")

    def _pipe(self):
        """A non-transactional redis-py pipeline -- one round trip for a whole batch
        of commands, executed in order -- when batching is on and the client has
        one; else None, and every command is its own round trip as in the
        reference (``:48-52``, ``:384``, ``:413``)."""
        if not self.batch_io:
            return None
        mk = getattr(self.redis_client, "pipeline", None)
        return mk(transaction=False) if mk is not None else None

    # ------------------------------------------------------------- slot mapping
    def _slot(self, worker_id):
        s = self.slot_of.get(worker_id)
        if s is not None:
            return s
        if self._free_slots:
            s = self._free_slots.pop()
        elif self._next_slot < self.max_workers:
            s = self._next_slot
            self._next_slot += 1
        else:
            raise FaasbalError(-1, "worker table full: %d slots (raise max_workers)" % self.max_workers)
        self.slot_of[worker_id] = s
        self.identity[s] = worker_id
        return s

    def _release(self, s):
        wid = self.identity[s]
        if wid is not None:
            del self.slot_of[wid]
            self.identity[s] = None
            self._free_slots.append(int(s))

    def _stamp(self):
        t = float(self.clock())
        if t < self._last_ts:  # the wall clock stepped back: keep the tick's stamps ordered
            t = self._last_ts
        self._last_ts = t
        return t

    # --------------------------------------------------------------------- ticks
    def _inbound_ready(self):
        return self.socket in dict(self.poller.poll(0))

    def _drain_inbound(self):
        msgs = []
        while len(msgs) < self.max_events and self._inbound_ready():
            worker_id, message = self.receive_message()
            msgs.append((worker_id, message, self._stamp()))
        return msgs

    def _drain_tasks(self):
        while True:
            m = self.subscriber.get_message()
            if m is None:
                break
            if m["type"] == "message":
                d = m["data"]
                self.pending.append(d.decode("utf-8") if isinstance(d, (bytes, bytearray)) else str(d))

    def tick(self):
        """One tick of the selected loop; returns the balancer's tick result dict."""
        msgs = self._drain_inbound()
        self._drain_tasks()
        return self._run(msgs)

    def _deque_filter(self, msgs):
        """start() (:271-295) acts on register and result only; a result from an
        identity without a record raises KeyError in the reference (after the
        HSET at :288).  Returns the messages for the balancer and the unknown
        results (kept out of the table, their HSET done here)."""
        keep, unknown = [], []
        known = set(self.slot_of)
        for wid, m, t in msgs:
            typ = m.get("type") if isinstance(m, dict) else None
            if typ == "register":
                known.add(wid)
                keep.append((wid, m, t))
            elif typ == "result":
                (keep if wid in known else unknown).append((wid, m, t))
        return keep, unknown

    def _run(self, msgs):
        # room for every dispatch this tick can make (orphans + pending) before sequence
        # numbers are taken.  Compaction reclaims the finished entries (head - in-flight);
        # when a backlog keeps the worst case above the log even after it, compacting
        # every tick would cost a full log round trip per tick while the dispatches are
        # bounded by the workers' free capacity -- so it runs then only when it reclaims a
        # quarter of the log, and the tick itself decides (a real overflow, FB_ENOSPC,
        # compacts and reruns the tick below).
        need = len(self.pending) + len(self.inflight)
        garbage = self.head - len(self.inflight)
        if self.head + need > self.max_inflight and garbage > 0 and (
                self.head - garbage + need <= self.max_inflight or 4 * garbage >= self.max_inflight):
            self.compact_log()
        now = self._stamp()
        arrived = msgs
        unknown = []
        if self.mode == "deque":
            msgs, unknown = self._deque_filter(msgs)
        E = len(msgs)
        kind = np.empty(E, np.uint8)
        slot = np.empty(E, np.int32)
        val = np.zeros(E, np.int32)
        ts = np.empty(E, np.float64)
        seq = np.full(E, -1, np.int64)
        for i, (wid, m, t) in enumerate(msgs):
            typ = m.get("type") if isinstance(m, dict) else None
            k = _KINDS.get(typ, EV_OTHER)
            kind[i] = k
            slot[i] = self._slot(wid)
            ts[i] = t
            if k == EV_REGISTER or k == EV_RECONNECT:
                v = int(m["data"]["num_processes" if k == EV_REGISTER else "free_processes"])
                if not (_I32[0] <= v <= _I32[1]):
                    raise FaasbalError(-1, "process count %d does not fit int32" % v)
                val[i] = v
            elif k == EV_RESULT:
                seq[i] = self.task_seq.get(m["data"]["task_id"], -1)
        # a one-GPU balancer hands the tick's assignments back in compact form -- slot and
        # min(c, L + 1) per LRU position, written by the tick into registered pinned arrays
        # (5 B per queued worker instead of 4 B per task) -- expanded round by round while the
        # task messages go out below; orphans / evicted slots in the same readback, consumed
        # before the next tick (exactly a GpuBalancer: a ShardedBalancer subclass has no pinned
        # path; shard groups are the sharded route)
        tkw = {"compact": True, "pinned": True} if type(self.balancer) is GpuBalancer else {}
        try:
            out = self.balancer.tick(now, float(self.time_to_expire), kind, slot, val, ts, seq,
                                     n_pending=len(self.pending), **tkw)
        except FaasbalError as e:
            # in-flight log full: the tick was not committed.  Compaction renumbers every
            # in-flight sequence, so the results' sequence numbers are looked up again
            # before the rerun; when nothing can be reclaimed the compaction still
            # reinstalls the device log from the host's view, then the error propagates.
            if e.code != FB_ENOSPC:
                raise
            reclaimable = self.head > len(self.inflight)
            self.compact_log()
            if not reclaimable:
                raise
            for i, (wid, m, t) in enumerate(msgs):
                if kind[i] == EV_RESULT:
                    seq[i] = self.task_seq.get(m["data"]["task_id"], -1)
            out = self.balancer.tick(now, float(self.time_to_expire), kind, slot, val, ts, seq,
                                     n_pending=len(self.pending), **tkw)
        res = out["result"]
        # ---- per-message replies, in arrival order (:356-358, :374-387; start(): :284-288,
        #      where a result from an unknown identity is still HSET before the KeyError)
        status = out["reconnect"]
        res["unknown_results"] = len(unknown)
        index = {id(x): i for i, x in enumerate(msgs)}
        has_results = any(isinstance(m, dict) and m.get("type") == "result" for _, m, _ in arrived)
        rpipe = self._pipe() if has_results else None
        rdb = rpipe if rpipe is not None else self.redis_client
        for x in arrived:
            wid, m, _ = x
            i = index.get(id(x))
            if i is None:  # deque loop: result from an identity without a record
                if m.get("type") == "result":
                    data = m["data"]
                    rdb.hset(data["task_id"], mapping={"status": data["status"], "result": data["result"]})
                continue
            if status[i] == FB_EVS_RECONNECT:
                self.send_message(wid, {"type": "reconnect"})
            elif kind[i] == EV_RESULT and status[i] == 0:
                data = m["data"]
                rdb.hset(data["task_id"], mapping={"status": data["status"], "result": data["result"]})
                q = int(seq[i])
                if q >= 0 and self.inflight.get(q, (None, -1))[1] == slot[i]:
                    tid, _ = self.inflight.pop(q)
                    self.task_seq.pop(tid, None)
        if rpipe is not None:
            rpipe.execute()
        # ---- redistribution: orphans (ascending old sequence) go first
        orphan_tids = []
        for q in out["orphans"]:
            tid, _ = self.inflight.pop(int(q))
            self.task_seq.pop(tid, None)
            orphan_tids.append(tid)
        if orphan_tids:
            self.pending.extendleft(reversed(orphan_tids))
        # ---- dispatch (:393-419): task k -> slot assign[k], log sequence base + k
        # Batched host I/O: the payload reads of the whole tick
        # in one pipeline round trip, the task messages, then the RUNNING writes in
        # one more -- the same commands, messages and writes in the same order as
        # the reference's per-task HGET, HGET, send, HSET (:398-413), 2 round trips
        # per tick instead of 3 per task.
        assign = out["assign"]
        n = int(res["n_assigned"])
        base = int(res["log_head"]) - n
        tids = [self.pending.popleft() for _ in range(n)]
        qpipe = self._pipe() if n else None
        if qpipe is not None:
            for tid in tids:
                qpipe.hget(tid, "fn_payload")
                qpipe.hget(tid, "param_payload")
            vals = qpipe.execute()
        wpipe = self._pipe() if n else None
        wdb = wpipe if wpipe is not None else self.redis_client
        # (the per-task slots in LRU rounds: a CompactAssignments expands as it is iterated)
        for k, (tid, s) in enumerate(zip(tids, assign)):
            s = int(s)
            if qpipe is None:
                task_id, fn_payload, param_payload = self.query_redis({"data": tid.encode("utf-8")})
            else:
                task_id, fn_payload, param_payload = tid, vals[2 * k].decode("utf-8"), vals[2 * k + 1].decode("utf-8")
            self.send_message(self.identity[s], {"type": "task", "data": {
                "task_id": task_id, "fn_payload": fn_payload, "param_payload": param_payload}})
            wdb.hset(task_id, mapping={"status": "RUNNING"})
            self.inflight[base + k] = (tid, s)
            self.task_seq[tid] = base + k
        if wpipe is not None:
            wpipe.execute()
        self.head = int(res["log_head"])
        # ---- evicted records: their identities become unknown (:246-249)
        for s in out["evicted"]:
            self._release(int(s))
        self.ticks += 1
        return res

    def start_heartbeat(self, max_ticks=None):
        """The dispatcher loop (``task_dispatcher.py:324-419``), one tick per pass."""
        self.use_loop("heartbeat")
        while max_ticks is None or self.ticks < max_ticks:
            self.tick()

    def start(self, max_ticks=None):
        """The loop without heartbeats (``task_dispatcher.py:251-322``), one tick per pass."""
        self.use_loop("deque")
        while max_ticks is None or self.ticks < max_ticks:
            self.tick()

    def purge_workers(self, free_workers=None):
        """``purge_workers`` (``:241-249``) on its own: records whose heartbeat expired
        at the current clock are deleted (their identities become unknown), nothing
        is dispatched and no message is sent.  The in-flight tasks of the dead
        workers -- which the reference loses (README.md:263-264) -- go to the front
        of the pending tasks, for the next tick's dispatch.  Returns the evicted
        identities."""
        out = self.balancer.purge(self._stamp(), float(self.time_to_expire))
        orphan_tids = []
        for q in out["orphans"]:
            tid, _ = self.inflight.pop(int(q))
            self.task_seq.pop(tid, None)
            orphan_tids.append(tid)
        if orphan_tids:
            self.pending.extendleft(reversed(orphan_tids))
        gone = [self.identity[int(s)] for s in out["evicted"]]
        for s in out["evicted"]:
            self._release(int(s))
        return gone

    # ------------------------------------------------------- state / inspection
    @property
    def workers(self):
        """``self.workers`` of the reference: identity -> PushWorker-like view (device read-back)."""
        st = self.balancer.read_state(with_log=False)
        return {wid: WorkerView(st["free"][s], st["hb"][s], self.time_to_expire)
                for wid, s in self.slot_of.items() if st["reg"][s]}

    @property
    def free_workers(self):
        """The LRU queue of the reference (``:327``; ``start()``: the deque of ``:254``,
        identities possibly repeated) as a list of identities, front first."""
        st = self.balancer.read_state(with_log=False)
        return [self.identity[s] for s in st["queue"]]

    def compact_log(self):
        """Renumber the in-flight log densely (completed and redistributed entries
        dropped); epochs are remapped so every registration keeps exactly its own
        in-flight entries.  Host O(F), called only when the log would overflow."""
        st = self.balancer.read_state(with_log=True)
        keep = np.asarray(sorted(self.inflight), np.int64)
        log = np.asarray([self.inflight[q][1] for q in keep], np.int32)
        epoch = np.searchsorted(keep, st["epoch"].astype(np.int64), side="left").astype(np.uint32)
        self.balancer.load_state(st["reg"], st["free"], st["hb"], epoch, st["queue"], log)
        remap = {int(q): i for i, q in enumerate(keep)}
        self.inflight = {remap[q]: v for q, v in self.inflight.items()}
        self.task_seq = {tid: remap[q] for tid, q in self.task_seq.items()}
        self.head = len(keep)
        self.compactions += 1

    def snapshot(self):
        """Host + device state (checkpoint; the reference keeps none)."""
        st = self.balancer.read_state(with_log=True)
        st.update(identity=list(self.identity), inflight=dict(self.inflight), pending=list(self.pending),
                  free_slots=list(self._free_slots), next_slot=self._next_slot)
        return st

    def restore(self, st):
        """Install a snapshot (or a hand-built state: reg/free/hb/epoch/queue/log plus
        identity[slot] and inflight{seq: (task_id, slot)})."""
        W = len(st["reg"])
        if W > self.max_workers:
            raise FaasbalError(-1, "snapshot has %d slots, table holds %d" % (W, self.max_workers))
        pad = self.max_workers - W
        reg = np.concatenate([np.asarray(st["reg"], np.uint8), np.zeros(pad, np.uint8)])
        free = np.concatenate([np.asarray(st["free"], np.int32), np.zeros(pad, np.int32)])
        hb = np.concatenate([np.asarray(st["hb"], np.float64), np.zeros(pad, np.float64)])
        ep = st.get("epoch")
        ep = np.zeros(W, np.uint32) if ep is None else np.asarray(ep, np.uint32)
        epoch = np.concatenate([ep, np.zeros(pad, np.uint32)])
        self.balancer.load_state(reg, free, hb, epoch, st["queue"], st["log"])
        self._reset_host()
        ident = list(st["identity"]) + [None] * (self.max_workers - len(st["identity"]))
        for s, wid in enumerate(ident):
            if wid is not None:
                self.slot_of[wid] = s
                self.identity[s] = wid
        self._next_slot = int(st.get("next_slot", max((s + 1 for s, w in enumerate(ident) if w is not None),
                                                      default=0)))
        used = set(self.slot_of.values())
        self._free_slots = list(st.get("free_slots", [s for s in range(self._next_slot) if s not in used][::-1]))
        self.inflight = {int(q): (tid, int(s)) for q, (tid, s) in st.get("inflight", {}).items()}
        self.task_seq = {tid: q for q, (tid, _) in self.inflight.items()}
        self.pending = collections.deque(st.get("pending", ()))
        self.head = len(st["log"])


def ShardedPushDispatcher(ip_address, port, time_to_expire=10, *, max_workers=65536, max_inflight=1 << 24,
                          max_events=65536, backend_balancer=None, **kw):
    """The heartbeat push dispatcher over a worker table sharded across the ranks of
    the current torch.distributed group (one process per GPU, RCCL over xGMI).

    Rank 0 gets a GpuPushDispatcher whose balancer is a DistShardGroup: it runs the
    ZMQ / Redis loop, broadcasts each tick's messages and pending count, every rank
    ticks its own slot range (exchange all-reduce in between) and rank 0 gathers the
    (task, slot) pairs and sends the task messages in ascending task order
    (task_dispatcher.py:409-413).  Ranks > 0 serve their shard and return None
    when rank 0 closes the group (``dispatcher.balancer.close()``)."""
    import torch.distributed as dist

    from .sharded import DistShardGroup, ShardedBalancer, serve_shard
    rank, world = dist.get_rank(), dist.get_world_size()
    bal = backend_balancer if backend_balancer is not None else \
        ShardedBalancer(rank, world, max_workers, max_inflight, max_events=max_events, device=kw.pop("device", 0))
    if rank != 0:
        serve_shard(bal)
        return None
    group = DistShardGroup(bal, max_workers)
    return GpuPushDispatcher(ip_address, port, time_to_expire, max_workers=max_workers, max_inflight=max_inflight,
                             max_events=max_events, balancer=group, **kw)
