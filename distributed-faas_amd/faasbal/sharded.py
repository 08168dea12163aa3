"""ShardedBalancer: one rank's share of a worker table split across GPUs.

The reference keeps every worker in one process (``self.workers`` dict and the
``free_workers`` OrderedDict, task_dispatcher.py:194, :327).  Here rank r of
``world`` owns the contiguous global slot range ``shard_range(W, world, r)``:
their records, their in-flight log entries and the dispatch of tasks to them.
The LRU queue order is replicated on every rank.  One tick is

    phase 1 (own slots: messages, purge, orphan flags, free counts)
    -> all-reduce(SUM) of a small uint8 exchange buffer over the ranks
    -> phase 2 (global water-filling from the exchanged counts; own writes)

and its whole-table result is bit-identical to the one-GPU tick.
The exchange buffer is a torch tensor so ``torch.distributed`` (RCCL over xGMI
on MI355X) can reduce it in place; the library runs on a torch stream that the
collective is issued on too, so kernels and collective are ordered on-device.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .balancer import GpuBalancer, _arr, _p
from ._lib import FB_ERERUN, FaasbalError

MAX_RELAUNCH = 6  # FB_ERERUN: each relaunch at least doubles the round table


def shard_range(n_workers, world, rank):
    """Global slot range [base, base + n) of ``rank``: contiguous blocks of ceil(W / world)."""
    per = -(-int(n_workers) // int(world))
    base = min(rank * per, n_workers)
    return base, min(per, n_workers - base)


def split_state(st, world, rank):
    """This rank's part of a global state dict (reg/free/hb/epoch/queue/log)."""
    W = len(st["reg"])
    base, n = shard_range(W, world, rank)
    log = np.asarray(st["log"], np.int32)
    seq = np.nonzero((log >= base) & (log < base + n))[0]
    epoch = st.get("epoch")
    epoch = np.zeros(W, np.uint32) if epoch is None else np.asarray(epoch, np.uint32)
    return dict(base=base, n=n, reg=np.asarray(st["reg"], np.uint8)[base:base + n],
                free=np.asarray(st["free"], np.int32)[base:base + n], hb=np.asarray(st["hb"], np.float64)[base:base + n],
                epoch=epoch[base:base + n], queue=np.asarray(st["queue"], np.int32), log_slot=log[seq],
                log_seq=seq.astype(np.uint32), log_head=len(log))


class ShardedBalancer(GpuBalancer):
    """Rank ``rank`` of ``world`` over a table of ``n_workers`` global slots."""

    def __init__(self, rank, world, n_workers, max_log, max_events=65536, device=0, lib_path=None):
        import torch  # the exchange buffer and the stream come from torch (plumbing, not compute)

        self.torch = torch
        self.rank, self.world, self.n_workers_global = int(rank), int(world), int(n_workers)
        self.base, self.n_local = shard_range(n_workers, world, rank)
        super().__init__(max(self.n_local, 1), max_log, max_events, device, lib_path)
        n = C.c_int64()
        self._chk(self.lib.fb_exchange_bytes(self.h, -1, C.byref(n)))
        self.xbuf = torch.zeros(n.value, dtype=torch.uint8, device="cuda:%d" % device)
        self._chk(self.lib.fb_bind_exchange(self.h, C.c_void_p(self.xbuf.data_ptr()), n.value))
        # kernels and the exchange collective share one torch stream (ordered, no host sync)
        self.stream = torch.cuda.Stream(device=device)
        self.set_stream(self.stream.cuda_stream)
        self._xbytes = 0

    def _create(self, max_workers, max_log, max_events, device):
        rc = self.lib.fb_create_sharded(C.byref(self.h), int(max_workers), self.n_workers_global, int(max_log),
                                        int(max_events), int(device), self.rank, self.world)
        if rc != 0:
            raise FaasbalError(rc, "fb_create_sharded(rank %d of %d, %d slots) failed"
                               % (self.rank, self.world, self.n_workers_global))

    # ----------------------------------------------------------------- state
    def load_state(self, *a, **k):
        raise FaasbalError(_lib.FB_ESTATE, "sharded context: use load() with the global state")

    def load(self, st):
        """Load this rank's part of a global state dict."""
        sh = split_state(st, self.world, self.rank)
        self._chk(self.lib.fb_load_shard(self.h, sh["base"], sh["n"], _p(sh["reg"]), _p(sh["free"]), _p(sh["hb"]),
                                         _p(sh["epoch"]), _p(sh["queue"]), len(sh["queue"]), _p(sh["log_slot"]),
                                         _p(sh["log_seq"]), len(sh["log_slot"]), sh["log_head"]))
        # the round table of the first tick from the GLOBAL max free count (every rank
        # computes it from the same global state, so the exchange layouts agree)
        q = np.asarray(st["queue"], np.int64)
        mf = int(np.asarray(st["free"])[q].max()) if len(q) else 1
        self._chk(self.lib.fb_set_round_hint(self.h, max(1, min(mf, 1 << 30))))
        self.n_workers = sh["n"]

    def read_state(self, with_log=True):
        out = super().read_state(with_log)
        n, head = C.c_int64(), C.c_int64()
        seq = np.zeros(max(len(out.get("log", ())), 1), np.uint32)
        self._chk(self.lib.fb_read_shard_log(self.h, _p(seq) if with_log else None, C.byref(n), C.byref(head)))
        out["head"] = head.value
        out["log_len"] = n.value
        if with_log:
            out["log_seq"] = seq[: n.value]
        out["base"] = self.base
        return out

    # ----------------------------------------------------------------- ticks
    def launch(self, *a, **k):
        """Phase 1.  Afterwards all-reduce ``exchange()`` (SUM) over the ranks, then ``cont()``."""
        super().launch(*a, **k)
        n = C.c_int64()
        self._chk(self.lib.fb_exchange_bytes(self.h, self._E, C.byref(n)))
        self._xbytes = n.value

    def exchange(self):
        """The tick's exchange region (a view of the bound torch tensor, kept while its size is)."""
        xv = getattr(self, "_xview", None)
        if xv is None or xv.numel() != self._xbytes:
            xv = self._xview = self.xbuf[: self._xbytes]
        return xv

    def cont(self):
        self._chk(self.lib.fb_tick_continue(self.h))

    def set_full_assign(self, on=True):
        """fb_set_full_assign: this rank's phase 2 also writes the whole tick's task -> slot
        array (assignments() then works here; the dispatcher's rank gathers no tasks)."""
        self._chk(self.lib.fb_set_full_assign(self.h, 1 if on else 0))
        self.full_assign = bool(on)

    def assignments(self, first=0, n=None):
        if not getattr(self, "full_assign", False):
            raise FaasbalError(_lib.FB_ESTATE, "sharded context: use local_assignments() (or set_full_assign)")
        return super().assignments(first, n)

    def _allreduce(self, allreduce):
        n = C.c_int64()
        self._chk(self.lib.fb_exchange_bytes(self.h, self._E, C.byref(n)))
        self._xbytes = n.value
        with self.torch.cuda.stream(self.stream):
            if allreduce is None:
                # issued on self.stream; the explicit wait orders phase 2 after it on that
                # stream (RCCL) or after its completion (gloo)
                self.torch.distributed.all_reduce(self.exchange(), async_op=True).wait()
            else:
                allreduce(self.exchange())

    def _run_phases(self, launch, allreduce):
        """Phase 1, the exchange, phase 2 and the wait -- again with a wider round table
        while the tick asks for it (FB_ERERUN: the same tick, relaunched; every rank
        gets the same answer, so the ranks' collectives stay matched)."""
        for attempt in range(MAX_RELAUNCH + 1):
            launch()
            self._allreduce(allreduce)
            self.cont()
            try:
                return self.wait()
            except FaasbalError as e:
                if e.code != FB_ERERUN or attempt == MAX_RELAUNCH:
                    raise

    def purge(self, now, tte, commit=True, allreduce=None):
        """This rank's share of ``purge_workers`` (``task_dispatcher.py:241-249``):
        the exchange and phase 2 run as for a tick, nothing is dispatched; returns
        dict(result, evicted, orphans) of this rank's slots and log shard."""
        self._E = 0
        res = self._run_phases(lambda: self._chk(self.lib.fb_purge_launch(self.h, float(now), float(tte))),
                               allreduce)
        out = dict(result=res, evicted=self.evicted(), orphans=self.orphans())
        if commit:
            self.commit()
        return out

    def tick(self, now, tte, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None, n_pending=0,
             commit=True, outputs=True, allreduce=None):
        """One sharded tick; ``allreduce(tensor)`` defaults to torch.distributed.all_reduce (SUM)."""
        res = self._run_phases(lambda: self.launch(now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, n_pending),
                               allreduce)
        out = dict(result=res)
        if outputs:
            # the whole tick's assignments where this rank writes them (set_full_assign), else
            # this rank's own (task, slot) pairs
            if getattr(self, "full_assign", False):
                out.update(assign=self.assignments())
            else:
                task, slot = self.local_assignments()
                out.update(task=task, slot=slot)
            out.update(reconnect=self.event_status(), orphans=self.orphans(), evicted=self.evicted())
        if commit:
            self.commit()
        return out


def merge_states(states, n_workers):
    """The global state (GpuBalancer.read_state layout) from every rank's read_state()."""
    reg = np.zeros(n_workers, np.uint8)
    free = np.zeros(n_workers, np.int32)
    hb = np.zeros(n_workers, np.float64)
    epoch = np.zeros(n_workers, np.uint32)
    for st in states:
        lo, n = st["base"], len(st["reg"])
        reg[lo:lo + n], free[lo:lo + n], hb[lo:lo + n], epoch[lo:lo + n] = st["reg"], st["free"], st["hb"], st["epoch"]
    head = states[0]["head"]
    out = dict(reg=reg, free=free, hb=hb, epoch=epoch, queue=np.asarray(states[0]["queue"], np.int32), head=head)
    if all("log" in st for st in states):
        log = np.full(head, -1, np.int32)
        for st in states:
            log[np.asarray(st["log_seq"], np.int64)] = st["log"]
        out["log"] = log
    return out


class ShardGroup:
    """A worker table sharded over ranks, behind GpuBalancer's tick API -- what
    GpuPushDispatcher drives (``balancer=``), so the drop-in's host loop, message
    flow and Redis I/O are the same for one GPU and for N.  Subclasses say how a
    call reaches the ranks: in this process (LocalShardGroup) or over
    torch.distributed from rank 0 (DistShardGroup)."""

    mode = "heartbeat"

    def __init__(self, n_workers):
        self.n_workers_global = int(n_workers)

    def _each(self, op, **kw):  # -> list of per-rank results, rank order
        raise NotImplementedError

    def load_state(self, reg, free, hb, epoch=None, queue=(), log=()):
        W = len(reg)
        st = dict(reg=np.asarray(reg, np.uint8), free=np.asarray(free, np.int32), hb=np.asarray(hb, np.float64),
                  epoch=np.zeros(W, np.uint32) if epoch is None else np.asarray(epoch, np.uint32),
                  queue=np.asarray(queue, np.int32), log=np.asarray(log, np.int32))
        self._each("load", st=st)

    def load(self, st):
        self.load_state(st["reg"], st["free"], st["hb"], st.get("epoch"), st["queue"], st["log"])

    def read_state(self, with_log=True):
        return merge_states(self._each("read", with_log=with_log), self.n_workers_global)

    def tick(self, now, tte, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None, n_pending=0):
        k = np.asarray(ev_kind, np.uint8)
        ev = dict(ev_kind=k, ev_slot=np.asarray(ev_slot, np.int32), ev_val=np.asarray(ev_val, np.int32),
                  ev_ts=np.asarray(ev_ts, np.float64),
                  ev_seq=np.full(len(k), -1, np.int64) if ev_seq is None else np.asarray(ev_seq, np.int64))
        outs = self._each("tick", now=float(now), tte=float(tte), n_pending=int(n_pending), **ev)
        res = dict(outs[0]["result"])
        for key in ("n_local", "n_orphans_local"):
            res[key] = sum(int(o["result"][key]) for o in outs)
        res["n_evicted"] = sum(int(o["result"]["n_evicted"]) for o in outs)
        merged = merge_outputs(outs, int(res["n_assigned"]))
        merged["result"] = res
        return merged

    def purge(self, now, tte):
        outs = self._each("purge", now=float(now), tte=float(tte))
        res = dict(outs[0]["result"])
        res["n_evicted"] = sum(int(o["result"]["n_evicted"]) for o in outs)
        return dict(result=res, evicted=np.sort(np.concatenate([o["evicted"] for o in outs])).astype(np.int32),
                    orphans=np.sort(np.concatenate([o["orphans"] for o in outs])).astype(np.int64))

    def close(self):
        pass


def serve_op(bal, op, kw, allreduce=None, commit=True):
    """One group operation on this rank's balancer (every rank runs the same op).
    ``commit=False`` leaves a tick / purge waited but uncommitted (DistShardGroup
    commits only once every rank has succeeded)."""
    if op == "load":
        bal.load(kw["st"])
        return None
    if op == "read":
        return bal.read_state(with_log=kw["with_log"])
    if op == "tick":
        out = bal.tick(kw["now"], kw["tte"], kw["ev_kind"], kw["ev_slot"], kw["ev_val"], kw["ev_ts"], kw["ev_seq"],
                       kw["n_pending"], allreduce=allreduce, commit=commit)
        return out
    if op == "purge":
        return bal.purge(kw["now"], kw["tte"], allreduce=allreduce, commit=commit)
    raise ValueError("unknown group operation %r" % op)


def _serve_guarded(bal, op, kw):
    """serve_op on this rank, its failure returned instead of raised: every rank must
    still reach the group's gather (a rank that skipped it would leave the others
    blocked in the collective).  A tick / purge is not committed here."""
    try:
        return (True, serve_op(bal, op, kw, commit=False))
    except Exception as e:  # noqa: BLE001 -- reported to rank 0, which raises it
        return (False, (getattr(e, "code", None), "%s: %s" % (type(e).__name__, e)))


def _settle(bal, op, outs):
    """After the gather, on every rank: commit a tick / purge only when it succeeded
    on every rank (so the shards never diverge); returns the first failure or None."""
    bad = next((o[1] for o in outs if not o[0]), None)
    if bad is None and op in ("tick", "purge"):
        bal.commit()
    return bad


# DistShardGroup's wire format per call: a fixed header tensor broadcast from rank 0
# (operation, event count, tasks, clock), then for ticks / purges the event batch packed
# into one byte tensor (25 B per message), and back a fixed header per rank (all
# gathered: every rank commits only when all succeeded) plus one padded byte tensor
# per rank gathered to rank 0 (tasks, slots, orphans, evicted).  Loads and state reads
# (not per tick) and failure messages travel as pickled objects.
_OP_CODES = {"tick": 1, "purge": 2, "load": 3, "read": 4, "stop": 5}
_OP_NAMES = {v: k for k, v in _OP_CODES.items()}
_HDR = 8  # int64 words of the call header / the per-rank result header


def _dev(dist):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def _pack_events(kw):
    k = np.ascontiguousarray(kw["ev_kind"], np.uint8)
    parts = [k.view(np.uint8), np.ascontiguousarray(kw["ev_slot"], np.int32).view(np.uint8),
             np.ascontiguousarray(kw["ev_val"], np.int32).view(np.uint8),
             np.ascontiguousarray(kw["ev_ts"], np.float64).view(np.uint8),
             np.ascontiguousarray(kw["ev_seq"], np.int64).view(np.uint8)]
    return np.concatenate(parts) if len(k) else np.zeros(0, np.uint8)


def _unpack_events(buf, E):
    o = [0, E, 5 * E, 9 * E, 17 * E, 25 * E]
    return dict(ev_kind=buf[o[0]:o[1]].copy(), ev_slot=buf[o[1]:o[2]].view(np.int32).copy(),
                ev_val=buf[o[2]:o[3]].view(np.int32).copy(), ev_ts=buf[o[3]:o[4]].view(np.float64).copy(),
                ev_seq=buf[o[4]:o[5]].view(np.int64).copy())


def _bcast_call(dist, dev, op, kw):
    """Rank 0: the call to every rank.  Returns nothing; the ranks read it with _recv_call."""
    import torch
    h = torch.zeros(_HDR, dtype=torch.int64)
    h[0] = _OP_CODES[op]
    if op in ("tick", "purge"):
        E = len(kw.get("ev_kind", ())) if op == "tick" else 0
        h[1] = E
        h[2] = int(kw.get("n_pending", 0))
        h[3] = int(np.float64(kw["now"]).view(np.int64))
        h[4] = int(np.float64(kw["tte"]).view(np.int64))
    dist.broadcast(h.to(dev), src=0)
    if op in ("tick", "purge"):
        if int(h[1]):
            dist.broadcast(torch.from_numpy(_pack_events(kw)).to(dev), src=0)
    elif op != "stop":
        dist.broadcast_object_list([kw], src=0)


def _recv_call(dist, dev):
    """Ranks > 0: the next call of rank 0 as (op, kw)."""
    import torch
    h = torch.zeros(_HDR, dtype=torch.int64, device=dev)
    dist.broadcast(h, src=0)
    h = h.cpu().numpy()
    op = _OP_NAMES[int(h[0])]
    if op not in ("tick", "purge"):
        if op == "stop":
            return op, {}
        box = [None]
        dist.broadcast_object_list(box, src=0)
        return op, box[0]
    E = int(h[1])
    kw = dict(now=float(h[3:4].view(np.float64)[0]), tte=float(h[4:5].view(np.float64)[0]), n_pending=int(h[2]))
    if op == "tick":
        if E:
            buf = torch.empty(25 * E, dtype=torch.uint8, device=dev)
            dist.broadcast(buf, src=0)
            kw.update(_unpack_events(buf.cpu().numpy(), E))
        else:
            z = np.zeros(0)
            kw.update(ev_kind=z.astype(np.uint8), ev_slot=z.astype(np.int32), ev_val=z.astype(np.int32),
                      ev_ts=z.astype(np.float64), ev_seq=z.astype(np.int64))
    return op, kw


def _gather_results(dist, dev, op, guarded):
    """Every rank: its guarded result of a tick / purge.  Returns, on every rank, the
    list of (ok, value | (code, message)) in rank order -- values complete on rank 0
    (the other ranks get headers only, enough to settle the commit)."""
    import torch
    ok, val = guarded
    rank, world = dist.get_rank(), dist.get_world_size()
    h = torch.zeros(_HDR, dtype=torch.int64)
    payload = np.zeros(0, np.uint8)
    if ok:
        r = val["result"]
        # (rank 0 writes the whole assignment array itself, fb_set_full_assign: the other
        # ranks send only their orphans and evicted slots, a few KB)
        task = np.zeros(0, np.int64)
        slot = np.zeros(0, np.int32)
        orph = np.asarray(val["orphans"], np.int64)
        evic = np.asarray(val["evicted"], np.int32)
        h[0] = 1
        h[2], h[3], h[4] = int(r.get("n_local", 0)), int(r.get("n_orphans_local", 0)), int(r["n_evicted"])
        h[5], h[6], h[7] = len(task), len(orph), len(evic)
        if rank != 0:
            payload = np.concatenate([task.view(np.uint8), slot.view(np.uint8), orph.view(np.uint8),
                                      evic.view(np.uint8)])
    else:
        h[1] = val[0] if val[0] is not None else 0
    hs = [torch.zeros(_HDR, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(hs, h.to(dev))
    hs = [x.cpu().numpy() for x in hs]
    if not all(x[0] for x in hs):
        # a rank failed: its message (pickled: failures only)
        msgs = [None] * world
        dist.all_gather_object(msgs, None if ok else val)
        return [(bool(x[0]), None if x[0] else msgs[i]) for i, x in enumerate(hs)]
    nbytes = [int(x[5]) * 12 + int(x[6]) * 8 + int(x[7]) * 4 for x in hs]
    mx = max(nbytes[1:], default=0)
    outs = [(True, val if rank == 0 else None)] + [(True, None)] * (world - 1)
    if world > 1 and mx > 0:
        mine = torch.zeros(mx, dtype=torch.uint8)
        if rank != 0:
            mine[:len(payload)] = torch.from_numpy(payload)
        bufs = [torch.zeros(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
        dist.gather(mine.to(dev), bufs, dst=0)
        if rank == 0:
            for i in range(1, world):
                b = bufs[i].cpu().numpy()
                nt, no, ne = int(hs[i][5]), int(hs[i][6]), int(hs[i][7])
                o = [0, 8 * nt, 12 * nt, 12 * nt + 8 * no, 12 * nt + 8 * no + 4 * ne]
                res = dict(n_local=int(hs[i][2]), n_orphans_local=int(hs[i][3]), n_evicted=int(hs[i][4]))
                d = dict(result=res, orphans=b[o[2]:o[3]].view(np.int64).copy(),
                         evicted=b[o[3]:o[4]].view(np.int32).copy(), reconnect=None)
                outs[i] = (True, d)
    elif rank == 0:
        for i in range(1, world):
            res = dict(n_local=int(hs[i][2]), n_orphans_local=int(hs[i][3]), n_evicted=int(hs[i][4]))
            d = dict(result=res, orphans=np.zeros(0, np.int64), evicted=np.zeros(0, np.int32), reconnect=None)
            outs[i] = (True, d)
    return outs


class DistShardGroup(ShardGroup):
    """Rank 0's view of a table sharded over a torch.distributed group (one process
    per GPU): every call is broadcast to the ranks (serve_shard() runs on the
    others), each rank runs it on its own shard -- ticks with the exchange
    all-reduce over the group's backend (RCCL over xGMI for ``nccl``) -- and the
    per-rank results come back to rank 0.  Ticks and purges travel as tensors (the
    event batch in one broadcast, the results in one gather); loads and state reads
    as pickled objects."""

    def __init__(self, balancer, n_workers):
        super().__init__(n_workers)
        import torch.distributed as dist
        self.dist, self.bal = dist, balancer
        if dist.get_rank() != 0:
            raise FaasbalError(_lib.FB_ESTATE, "DistShardGroup lives on rank 0; run serve_shard() on the others")
        self.dev = _dev(dist)
        # rank 0's phase 2 writes the whole assignment array (the per-task gather is gone)
        balancer.set_full_assign(True)

    def _each(self, op, **kw):
        _bcast_call(self.dist, self.dev, op, kw)
        guarded = _serve_guarded(self.bal, op, kw)
        if op in ("tick", "purge"):
            outs = _gather_results(self.dist, self.dev, op, guarded)
        else:
            outs = [None] * self.dist.get_world_size()
            self.dist.all_gather_object(outs, guarded)
        bad = _settle(self.bal, op, outs)
        if bad is not None:
            code, msg = bad
            if code is None:
                raise RuntimeError("shard operation %r failed on a rank: %s" % (op, msg))
            raise FaasbalError(code, "shard operation %r failed on a rank: %s" % (op, msg))
        return [o[1] for o in outs]

    def close(self):
        _bcast_call(self.dist, self.dev, "stop", {})


def serve_shard(balancer):
    """Rank r > 0 of a DistShardGroup: run rank 0's calls on this shard until it stops."""
    import torch.distributed as dist
    dev = _dev(dist)
    while True:
        op, kw = _recv_call(dist, dev)
        if op == "stop":
            return
        guarded = _serve_guarded(balancer, op, kw)
        if op in ("tick", "purge"):
            outs = _gather_results(dist, dev, op, guarded)
        else:
            outs = [None] * dist.get_world_size()
            dist.all_gather_object(outs, guarded)
        _settle(balancer, op, outs)  # rank 0 raises a failure; this rank keeps serving


class LocalShardGroup(ShardGroup):
    """Every rank's shard in this process (one GPU, or rank contexts on several
    devices); the exchange is summed on the device -- the reduction RCCL performs
    across GPUs, byte for byte (one contributor per byte)."""

    def __init__(self, world, n_workers, max_log, max_events=65536, device=0, rank_factory=None):
        super().__init__(n_workers)
        make = rank_factory or (lambda r: ShardedBalancer(r, world, n_workers, max_log, max_events, device))
        self.bals = [make(r) for r in range(world)]

    def _each(self, op, **kw):
        if op in ("tick", "purge"):
            return self._collective(op, kw)
        return [serve_op(b, op, kw) for b in self.bals]

    def _collective(self, op, kw):
        # phase 1 on every rank, then the summed exchange, then phase 2 / outputs / commit;
        # relaunched with a wider round table while the ranks ask for it (FB_ERERUN)
        for attempt in range(MAX_RELAUNCH + 1):
            try:
                return self._collective_once(op, kw)
            except FaasbalError as e:
                if e.code != FB_ERERUN or attempt == MAX_RELAUNCH:
                    raise

    def _collective_once(self, op, kw):
        torch = self.bals[0].torch
        for b in self.bals:
            if op == "tick":
                b.launch(kw["now"], kw["tte"], kw["ev_kind"], kw["ev_slot"], kw["ev_val"], kw["ev_ts"], kw["ev_seq"],
                         kw["n_pending"])
            else:
                b._E = 0
                b._chk(b.lib.fb_purge_launch(b.h, kw["now"], kw["tte"]))
                n = C.c_int64()
                b._chk(b.lib.fb_exchange_bytes(b.h, 0, C.byref(n)))
                b._xbytes = n.value
        torch.cuda.synchronize()
        total = self.bals[0].exchange().clone()
        for b in self.bals[1:]:
            total += b.exchange()
        for b in self.bals:
            b.exchange().copy_(total)
        torch.cuda.synchronize()
        for b in self.bals:
            b.cont()
        res_all = []
        err = None
        for b in self.bals:  # every rank waits (a rerun request reaches them all)
            try:
                res_all.append(b.wait())
            except FaasbalError as e:
                err = err or e
        if err is not None:
            raise err
        outs = []
        for b, res in zip(self.bals, res_all):
            if op == "tick":
                task, slot = b.local_assignments()
                outs.append(dict(result=res, task=task, slot=slot, orphans=b.orphans(), evicted=b.evicted(),
                                 reconnect=b.event_status()))
            else:
                outs.append(dict(result=res, evicted=b.evicted(), orphans=b.orphans()))
        for b in self.bals:
            b.commit()
        return outs

    def close(self):
        for b in self.bals:
            b.close()


def merge_outputs(outs, n_assigned):
    """Whole-table outputs from every rank's tick outputs (test / host-side helper): the
    assignment array of a rank that wrote it whole (set_full_assign), else the union of
    the ranks' (task, slot) pairs."""
    full = next((o["assign"] for o in outs if o.get("assign") is not None), None)
    if full is not None:
        assign = np.asarray(full, np.int32)
    else:
        assign = np.full(n_assigned, -1, np.int32)
        for o in outs:
            assign[o["task"]] = o["slot"]
    orphans = np.sort(np.concatenate([o["orphans"] for o in outs])) if outs else np.zeros(0, np.int64)
    evicted = np.sort(np.concatenate([o["evicted"] for o in outs])) if outs else np.zeros(0, np.int32)
    return dict(reconnect=outs[0]["reconnect"], assign=assign, orphans=orphans.astype(np.int64),
                evicted=evicted.astype(np.int32))
