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
from ._lib import FaasbalError


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

    def tick(self, now, tte, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None, n_pending=0,
             commit=True, outputs=True, allreduce=None):
        """One sharded tick; ``allreduce(tensor)`` defaults to torch.distributed.all_reduce (SUM)."""
        self.launch(now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, n_pending)
        with self.torch.cuda.stream(self.stream):
            if allreduce is None:
                # issued on self.stream; the explicit wait orders phase 2 after it on that
                # stream (RCCL) or after its completion (gloo)
                self.torch.distributed.all_reduce(self.exchange(), async_op=True).wait()
            else:
                allreduce(self.exchange())
        self.cont()
        res = self.wait()
        out = dict(result=res)
        if outputs:
            task, slot = self.local_assignments()
            out.update(reconnect=self.event_status(), task=task, slot=slot, orphans=self.orphans(),
                       evicted=self.evicted())
        if commit:
            self.commit()
        return out


def merge_outputs(outs, n_assigned):
    """Whole-table outputs from every rank's tick outputs (test / host-side helper)."""
    assign = np.full(n_assigned, -1, np.int32)
    for o in outs:
        assign[o["task"]] = o["slot"]
    orphans = np.sort(np.concatenate([o["orphans"] for o in outs])) if outs else np.zeros(0, np.int64)
    evicted = np.sort(np.concatenate([o["evicted"] for o in outs])) if outs else np.zeros(0, np.int32)
    return dict(reconnect=outs[0]["reconnect"], assign=assign, orphans=orphans.astype(np.int64),
                evicted=evicted.astype(np.int32))
