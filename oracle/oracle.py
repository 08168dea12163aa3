"""ctypes wrapper around oracle/build/libfaas_oracle.so -- TEST INFRASTRUCTURE ONLY.

The C restatement (``push_oracle.c``) follows the reference loop
``PushDispatcher.start_heartbeat`` (reference ``task_dispatcher.py:324-419``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module; the product (``faasbal``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libfaas_oracle.so")

_P = C.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _lib():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    lib.oracle_create.restype = _P
    lib.oracle_create.argtypes = [C.c_int32, C.c_int64]
    lib.oracle_destroy.argtypes = [_P]
    lib.oracle_set_purge_mode.argtypes = [_P, C.c_int]
    lib.oracle_load.restype = C.c_int
    lib.oracle_load.argtypes = [_P, _P, _P, _P, _P, _P, C.c_int64, _P, C.c_int64]
    lib.oracle_export.restype = C.c_int64
    lib.oracle_export.argtypes = [_P] * 8
    lib.oracle_tick.restype = C.c_int
    lib.oracle_tick.argtypes = [_P, C.c_double, C.c_double, C.c_int32, _P, _P, _P, _P, _P,
                                C.c_int64, C.c_int64, _P, _P, _P, _P, _P, _P, _P]
    lib.dq_oracle_create.restype = _P
    lib.dq_oracle_create.argtypes = [C.c_int32, C.c_int64]
    lib.dq_oracle_destroy.argtypes = [_P]
    lib.dq_oracle_load.restype = C.c_int
    lib.dq_oracle_load.argtypes = [_P, _P, _P, _P, _P, C.c_int64, _P, C.c_int64]
    lib.dq_oracle_export.restype = C.c_int64
    lib.dq_oracle_export.argtypes = [_P] * 7
    lib.dq_oracle_tick.restype = C.c_int
    lib.dq_oracle_tick.argtypes = [_P, C.c_int32, _P, _P, _P, _P, _P, C.c_int64, C.c_int64, _P, _P, _P]
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _lib()
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


class Oracle:
    """Sequential CPU restatement of the reference loop (purge_mode 0 = O(W)
    purge every iteration exactly as written; 1 = skip provably idempotent
    repeats, same results)."""

    def __init__(self, W, log_cap, purge_mode=1):
        self.W = int(W)
        self.log_cap = int(log_cap)
        self.h = lib().oracle_create(self.W, self.log_cap)
        if not self.h:
            raise MemoryError("oracle_create failed")
        lib().oracle_set_purge_mode(self.h, int(purge_mode))

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            lib().oracle_destroy(h)
            self.h = None

    def load(self, reg, free, hb, epoch, queue, log):
        reg = np.ascontiguousarray(reg, np.uint8)
        free = np.ascontiguousarray(free, np.int32)
        hb = np.ascontiguousarray(hb, np.float64)
        epoch = np.ascontiguousarray(epoch, np.uint32)
        queue = np.ascontiguousarray(queue, np.int32)
        log = np.ascontiguousarray(log, np.int32)
        rc = lib().oracle_load(self.h, _ptr(reg), _ptr(free), _ptr(hb), _ptr(epoch),
                               _ptr(queue), len(queue), _ptr(log), len(log))
        if rc != 0:
            raise ValueError("inconsistent state")

    def export(self):
        W = self.W
        reg = np.zeros(W, np.uint8)
        free = np.zeros(W, np.int32)
        hb = np.zeros(W, np.float64)
        epoch = np.zeros(W, np.uint32)
        queue = np.zeros(W, np.int32)
        log = np.zeros(self.log_cap, np.int32)
        head = np.zeros(1, np.int64)
        n = lib().oracle_export(self.h, _ptr(reg), _ptr(free), _ptr(hb), _ptr(epoch),
                                _ptr(queue), _ptr(log), _ptr(head))
        return dict(reg=reg, free=free, hb=hb, epoch=epoch, queue=queue[:n],
                    log=log[: int(head[0])], head=int(head[0]))

    def tick(self, now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, n_pending,
             dispatch_limit=-1, orphan_cap=None):
        E = len(ev_kind)
        ev_kind = np.ascontiguousarray(ev_kind, np.uint8)
        ev_slot = np.ascontiguousarray(ev_slot, np.int32)
        ev_val = np.ascontiguousarray(ev_val, np.int32)
        ev_ts = np.ascontiguousarray(ev_ts, np.float64)
        ev_seq = np.ascontiguousarray(ev_seq, np.int64)
        rec = np.zeros(max(E, 1), np.uint8)
        head = self.export_head()
        ocap = head if orphan_cap is None else orphan_cap
        orph = np.zeros(max(ocap, 1), np.int64)
        cap_assign = max(0, self.log_cap - head)
        assign = np.zeros(max(cap_assign, 1), np.int32)
        ev = np.zeros(max(self.W, 1), np.int32)
        na = np.zeros(1, np.int64)
        no = np.zeros(1, np.int64)
        ne = np.zeros(1, np.int32)
        rc = lib().oracle_tick(self.h, float(now), float(tte), E, _ptr(ev_kind), _ptr(ev_slot),
                               _ptr(ev_val), _ptr(ev_ts), _ptr(ev_seq), int(n_pending),
                               int(dispatch_limit), _ptr(rec), _ptr(assign), _ptr(na),
                               _ptr(orph), _ptr(no), _ptr(ev), _ptr(ne))
        if rc != 0:
            raise RuntimeError("oracle log overflow")
        return dict(reconnect=rec[:E].copy(), assign=assign[: int(na[0])].copy(),
                    orphans=orph[: int(no[0])].copy(), evicted=ev[: int(ne[0])].copy())

    def export_head(self):
        head = np.zeros(1, np.int64)
        lib().oracle_export(self.h, None, None, None, None, None, None, _ptr(head))
        return int(head[0])


class DequeOracle:
    """Sequential CPU restatement of the reference's ``PushDispatcher.start``
    (``task_dispatcher.py:251-322``): no heartbeats, a deque that may repeat ids
    (``deque_oracle.c``).  Same call shape as :class:`Oracle`; ``now``/``tte``
    are accepted and unused (start() has no liveness).  Event status in
    ``reconnect``: 2 = result from an id without a record (KeyError in the
    reference)."""

    def __init__(self, W, log_cap):
        self.W = int(W)
        self.log_cap = int(log_cap)
        self.h = lib().dq_oracle_create(self.W, self.log_cap)
        if not self.h:
            raise MemoryError("dq_oracle_create failed")

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            lib().dq_oracle_destroy(h)
            self.h = None

    def load(self, reg, free, hb, epoch, queue, log):
        del epoch  # no redistribution without heartbeats
        reg = np.ascontiguousarray(reg, np.uint8)
        free = np.ascontiguousarray(free, np.int32)
        hb = np.ascontiguousarray(hb, np.float64)
        queue = np.ascontiguousarray(queue, np.int32)
        log = np.ascontiguousarray(log, np.int32)
        if lib().dq_oracle_load(self.h, _ptr(reg), _ptr(free), _ptr(hb), _ptr(queue), len(queue), _ptr(log),
                                len(log)) != 0:
            raise ValueError("inconsistent state")

    def export(self):
        W = self.W
        reg = np.zeros(W, np.uint8)
        free = np.zeros(W, np.int32)
        hb = np.zeros(W, np.float64)
        head = np.zeros(1, np.int64)
        n = lib().dq_oracle_export(self.h, None, None, None, None, None, _ptr(head))
        queue = np.zeros(max(n, 1), np.int32)
        log = np.zeros(max(int(head[0]), 1), np.int32)
        lib().dq_oracle_export(self.h, _ptr(reg), _ptr(free), _ptr(hb), _ptr(queue), _ptr(log), _ptr(head))
        return dict(reg=reg, free=free, hb=hb, epoch=np.zeros(W, np.uint32), queue=queue[:n],
                    log=log[: int(head[0])], head=int(head[0]))

    def tick(self, now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, n_pending, dispatch_limit=-1):
        del now, tte
        E = len(ev_kind)
        ev_kind = np.ascontiguousarray(ev_kind, np.uint8)
        ev_slot = np.ascontiguousarray(ev_slot, np.int32)
        ev_val = np.ascontiguousarray(ev_val, np.int32)
        ev_ts = np.ascontiguousarray(ev_ts, np.float64)
        ev_seq = np.ascontiguousarray(ev_seq, np.int64)
        status = np.zeros(max(E, 1), np.uint8)
        head = np.zeros(1, np.int64)
        lib().dq_oracle_export(self.h, None, None, None, None, None, _ptr(head))
        assign = np.zeros(max(self.log_cap - int(head[0]), 1), np.int32)
        na = np.zeros(1, np.int64)
        rc = lib().dq_oracle_tick(self.h, E, _ptr(ev_kind), _ptr(ev_slot), _ptr(ev_val), _ptr(ev_ts), _ptr(ev_seq),
                                  int(n_pending), int(dispatch_limit), _ptr(status), _ptr(assign), _ptr(na))
        if rc != 0:
            raise RuntimeError("deque oracle: log overflow" if rc == -1 else "deque oracle: out of memory")
        return dict(reconnect=status[:E].copy(), assign=assign[: int(na[0])].copy(),
                    orphans=np.zeros(0, np.int64), evicted=np.zeros(0, np.int32))


def fixture_ticks(z):
    """Yield per-tick input dicts from a golden npz (events with resolved seqs)."""
    off = z["ev_off"]
    for t in range(int(z["n_ticks"])):
        a, b = int(off[t]), int(off[t + 1])
        yield dict(now=float(z["now"][t]), n_new=int(z["n_new"][t]),
                   ev_kind=z["ev_kind"][a:b], ev_slot=z["ev_slot"][a:b], ev_val=z["ev_val"][a:b],
                   ev_ts=z["ev_ts"][a:b], ev_seq=z["ev_seq"][a:b])


def fixture_expect(z, t):
    sl = lambda key: z["exp_" + key][int(z["exp_%s_off" % key][t]): int(z["exp_%s_off" % key][t + 1])]
    off = z["ev_off"]
    return dict(reconnect=z["exp_reconnect"][int(off[t]): int(off[t + 1])],
                assign=sl("assign"), orphans=sl("orphan"), evicted=sl("evicted"),
                n_pending=int(z["exp_n_pending"][t]),
                post_reg=z["exp_post_reg"][t], post_free=z["exp_post_free"][t],
                post_hb=z["exp_post_hb"][t], post_queue=sl("post_queue"))
