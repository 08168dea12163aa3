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
        """The tick's exchange region (a view of the bound torch tensor)."""
        return self.xbuf[: self._xbytes]

    def cont(self):
        self._chk(self.lib.fb_tick_continue(self.h))

    def assignments(self, first=0, n=None):
        raise FaasbalError(_lib.FB_ESTATE, "sharded context: use local_assignments()")

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
            task, slot = self.local_assignments()
            out.update(reconnect=self.event_status(), task=task, slot=slot, orphans=self.orphans(),
                       evicted=self.evicted())
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


class DistShardGroup(ShardGroup):
    """Rank 0's view of a table sharded over a torch.distributed group (one process
    per GPU): every call is broadcast to the ranks (serve_shard() runs on the
    others), each rank runs it on its own shard -- ticks with the exchange
    all-reduce over the group's backend (RCCL over xGMI for ``nccl``) -- and the
    per-rank results come back through one all_gather_object."""

    def __init__(self, balancer, n_workers):
        super().__init__(n_workers)
        import torch.distributed as dist
        self.dist, self.bal = dist, balancer
        if dist.get_rank() != 0:
            raise FaasbalError(_lib.FB_ESTATE, "DistShardGroup lives on rank 0; run serve_shard() on the others")

    def _each(self, op, **kw):
        self.dist.broadcast_object_list([(op, kw)], src=0)
        outs = [None] * self.dist.get_world_size()
        self.dist.all_gather_object(outs, _serve_guarded(self.bal, op, kw))
        bad = _settle(self.bal, op, outs)
        if bad is not None:
            code, msg = bad
            if code is None:
                raise RuntimeError("shard operation %r failed on a rank: %s" % (op, msg))
            raise FaasbalError(code, "shard operation %r failed on a rank: %s" % (op, msg))
        return [o[1] for o in outs]

    def close(self):
        self.dist.broadcast_object_list([("stop", {})], src=0)


def serve_shard(balancer):
    """Rank r > 0 of a DistShardGroup: run rank 0's calls on this shard until it stops."""
    import torch.distributed as dist
    while True:
        box = [None]
        dist.broadcast_object_list(box, src=0)
        op, kw = box[0]
        if op == "stop":
            return
        outs = [None] * dist.get_world_size()
        dist.all_gather_object(outs, _serve_guarded(balancer, op, kw))
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
    """Whole-table outputs from every rank's tick outputs (test / host-side helper)."""
    assign = np.full(n_assigned, -1, np.int32)
    for o in outs:
        assign[o["task"]] = o["slot"]
    orphans = np.sort(np.concatenate([o["orphans"] for o in outs])) if outs else np.zeros(0, np.int64)
    evicted = np.sort(np.concatenate([o["evicted"] for o in outs])) if outs else np.zeros(0, np.int32)
    return dict(reconnect=outs[0]["reconnect"], assign=assign, orphans=orphans.astype(np.int64),
                evicted=evicted.astype(np.int32))
