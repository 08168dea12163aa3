"""GpuBalancer: Python handle on one libfaasbal context (one GPU, one stream).

One ``tick`` replaces, for a batch of inbound messages and pending tasks, the
work that ``PushDispatcher.start_heartbeat`` (reference
``task_dispatcher.py:324-419``) does message by message: the inbound branches
(:343-387), ``purge_workers`` (:241-249, called at :390) and the LRU dispatch
block (:393-419), plus redistribution of the dead workers' in-flight tasks.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

import numpy as np

from . import _lib
from ._lib import FaasbalError, TickResult

_NONE = None

# Test paths (fb_set_path) applied to every context created in this process: the
# launch sequences of other table sizes on small, oracle-checkable inputs.  Test
# fixtures set them (tests/test_gpu_parity.py); production code leaves this empty.
TEST_PATHS = {}
# ... or from the environment for same-box A/B runs (tools/ab_stream.sh):
# FAASBAL_PATHS="cmix=0,wtiles=2".  Only knobs that leave the sharded exchange layout alone
# (a per-process value of one that changes it, e.g. xplan, would split a group's ranks);
# a malformed entry is reported, not fatal to the import.
_ENV_PATHS_REFUSED = ("xplan",)


def _env_paths(spec):
    out = {}
    for kv in filter(None, (x.strip() for x in spec.split(","))):
        k, sep, v = kv.partition("=")
        k = k.strip()
        try:
            val = int(v)
        except ValueError:
            val = None
        if not sep or not k or val is None:
            import warnings
            warnings.warn("FAASBAL_PATHS: ignoring %r (expected name=integer)" % kv)
            continue
        if k in _ENV_PATHS_REFUSED:
            import warnings
            warnings.warn("FAASBAL_PATHS: ignoring %r (it changes the sharded exchange layout; set it with "
                          "fb_set_path on every rank)" % kv)
            continue
        out[k] = val
    return out


TEST_PATHS.update(_env_paths(os.environ.get("FAASBAL_PATHS", "")))


def iter_compact(slot, c, n):
    """The per-task slots of a tick (``assignments()``) from its compact form, one LRU
    round at a time: round r serves, in LRU order, the positions whose min(c, L + 1) > r
    (``task_dispatcher.py:393-419`` in closed form), the last round only
    its first p.  Yields int32 arrays whose concatenation is the first ``n`` tasks' slots;
    each round filters the one before it, so the whole walk touches every task once."""
    sl = np.asarray(slot, np.int32)
    cc = np.asarray(c, np.uint8)
    r, left = 0, int(n)
    while left > 0:
        keep = cc > r
        sl, cc = sl[keep], cc[keep]
        if not len(sl):
            raise ValueError("compact form holds fewer than %d tasks" % n)
        take = sl[:left]
        left -= len(take)
        yield take
        r += 1


class CompactAssignments:
    """A tick's task -> slot assignments held in compact form (slot and min(c, L + 1) per
    LRU position, 5 bytes per queued worker instead of 4 per task): iterating yields the
    slot of task 0, 1, ... expanded round by round as the consumer goes
    (``GpuPushDispatcher`` sends while it expands); ``array()`` expands it whole."""

    def __init__(self, slot, c, n):
        self.slot, self.c, self.n = slot, c, int(n)

    def __len__(self):
        return self.n

    def chunks(self):
        return iter_compact(self.slot, self.c, self.n)

    def __iter__(self):
        for ch in self.chunks():
            yield from ch.tolist()

    def array(self):
        return np.concatenate(list(self.chunks())) if self.n else np.zeros(0, np.int32)


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


def _arr(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class GpuBalancer:
    """Device-resident worker table + LRU queue + in-flight log on one GPU.

    ``mode="heartbeat"`` (default) runs ``PushDispatcher.start_heartbeat``
    (``task_dispatcher.py:324-419``) per tick; ``mode="deque"`` runs the loop
    without heartbeats, ``PushDispatcher.start`` (``:251-322``), whose ready
    queue is a deque that may repeat ids (capacity ``max_tokens``, default
    ``2 * max_workers + max_events``)."""

    def __init__(self, max_workers, max_log, max_events=65536, device=0, lib_path=None, mode="heartbeat",
                 max_tokens=None):
        if mode not in ("heartbeat", "deque"):
            raise ValueError("mode must be 'heartbeat' or 'deque'")
        self.lib = _lib.load() if lib_path is None else _lib.load(lib_path)
        self.h = C.c_void_p()
        self.mode = mode
        if mode == "deque":
            self.max_tokens = int(max_tokens if max_tokens is not None else 2 * max_workers + max(max_events, 1))
            rc = self.lib.fb_create_deque(C.byref(self.h), int(max_workers), self.max_tokens, int(max_log),
                                          int(max_events), int(device))
            if rc != 0:
                raise FaasbalError(rc, "fb_create_deque(max_workers=%d, max_tokens=%d, max_log=%d, max_events=%d, "
                                       "device=%d) failed" % (max_workers, self.max_tokens, max_log, max_events,
                                                              device))
        else:
            self._create(max_workers, max_log, max_events, device)
        self.device = int(device)
        self.max_workers = int(max_workers)
        self.max_log = int(max_log)
        self.max_events = int(max_events)
        self.n_workers = 0
        self._E = 0
        for name, value in TEST_PATHS.items():
            self.set_path(name, value)

    def set_path(self, name, value):
        """fb_set_path: run another table size's launch sequence (results are identical)."""
        self._chk(self.lib.fb_set_path(self.h, name.encode(), int(value)))

    def _create(self, max_workers, max_log, max_events, device):
        rc = self.lib.fb_create(C.byref(self.h), int(max_workers), int(max_log), int(max_events), int(device))
        if rc != 0:
            raise FaasbalError(rc, "fb_create(max_workers=%d, max_log=%d, max_events=%d, device=%d) failed"
                               % (max_workers, max_log, max_events, device))

    # ------------------------------------------------------------------ misc
    def _chk(self, rc):
        if rc != 0:
            msg = self.lib.fb_last_error(self.h)
            raise FaasbalError(rc, msg.decode() if msg else "")

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.lib.fb_destroy(self.h)
            self.h = C.c_void_p()

    def pinned(self, n, dtype=np.int32):
        """A numpy array in pinned host memory: output copies into it
        (``assignments(out=...)``) are single transfers.  The memory is freed when the
        last array viewing it is collected -- not with the context, so an array that
        outlives ``close()`` never points at freed memory."""
        dtype = np.dtype(dtype)
        p = C.c_void_p()
        self._chk(self.lib.fb_host_alloc(self.h, int(n) * dtype.itemsize, C.byref(p)))
        buf = (C.c_char * max(int(n) * dtype.itemsize, 1)).from_address(p.value)
        # buf is the base of every view of the array; fb_host_free(NULL, p) needs no context
        weakref.finalize(buf, self.lib.fb_host_free, None, C.c_void_p(p.value))
        return np.frombuffer(buf, dtype=dtype, count=int(n))

    def pin_events(self, ev_kind, ev_slot, ev_val, ev_ts, ev_seq=None):
        """Copies of a tick's message arrays in pinned host memory: ``stage()`` of
        pinned arrays validates them in place and the H2D copies read them directly
        (no staging copy); they must stay unchanged until that tick was waited for."""
        out = []
        for a, dt in ((ev_kind, np.uint8), (ev_slot, np.int32), (ev_val, np.int32), (ev_ts, np.float64),
                      (ev_seq, np.int64)):
            if a is None:
                out.append(None)
                continue
            a = np.asarray(a, dt)
            b = self.pinned(len(a), dt)
            b[:] = a
            out.append(b)
        return out

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ----------------------------------------------------------------- state
    def load_state(self, reg, free, hb, epoch=None, queue=(), log=()):
        reg = _arr(reg, np.uint8)
        W = len(reg)
        free = _arr(free, np.int32)
        hb = _arr(hb, np.float64)
        epoch = _arr(np.zeros(W, np.uint32) if epoch is None else epoch, np.uint32)
        queue = _arr(queue, np.int32)
        log = _arr(log, np.int32)
        assert len(free) == W and len(hb) == W and len(epoch) == W
        self._chk(self.lib.fb_load_state(self.h, W, _p(reg), _p(free), _p(hb), _p(epoch), _p(queue),
                                         len(queue), _p(log), len(log)))
        self.n_workers = W

    def load(self, st):
        """Load a dict as produced by faasbal.synth (reg/free/hb/epoch/queue/log)."""
        self.load_state(st["reg"], st["free"], st["hb"], st.get("epoch"), st["queue"], st["log"])

    def read_state(self, with_log=True):
        W = self.n_workers
        qlen = C.c_int64()
        loglen = C.c_int64()
        self._chk(self.lib.fb_read_state(self.h, None, None, None, None, None, C.byref(qlen), None,
                                         C.byref(loglen)))
        reg = np.zeros(max(W, 1), np.uint8)
        free = np.zeros(max(W, 1), np.int32)
        hb = np.zeros(max(W, 1), np.float64)
        epoch = np.zeros(max(W, 1), np.uint32)
        queue = np.zeros(max(qlen.value, 1), np.int32)
        log = np.zeros(max(loglen.value, 1), np.int32) if with_log else None
        self._chk(self.lib.fb_read_state(self.h, _p(reg), _p(free), _p(hb), _p(epoch), _p(queue),
                                         C.byref(qlen), _p(log) if with_log else None, C.byref(loglen)))
        out = dict(reg=reg[:W], free=free[:W], hb=hb[:W], epoch=epoch[:W], queue=queue[: qlen.value],
                   head=loglen.value)
        if with_log:
            out["log"] = log[: loglen.value]
        return out

    def inflight(self):
        """Per-slot count of in-flight log entries (committed state; one-GPU heartbeat)."""
        out = np.zeros(max(self.n_workers, 1), np.uint32)
        self._chk(self.lib.fb_read_inflight(self.h, _p(out)))
        return out[: self.n_workers]

    # ----------------------------------------------------------------- ticks
    def launch(self, now, tte, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None, n_pending=0):
        if not len(ev_kind) and not len(ev_slot):
            # a tick without messages (the common idle / dispatch-only tick): straight to
            # the C ABI, no array conversions (they cost more host time than the launch)
            self._E = 0
            rc = self.lib.fb_tick_launch(self.h, now, tte, 0, None, None, None, None, None, n_pending)
            if rc:
                self._chk(rc)
            return
        k = _arr(ev_kind, np.uint8)
        s = _arr(ev_slot, np.int32)
        v = _arr(ev_val, np.int32)
        t = _arr(ev_ts, np.float64)
        q = None if ev_seq is None else _arr(ev_seq, np.int64)
        E = len(k)
        if not (len(s) == E and len(v) == E and len(t) == E and (q is None or len(q) == E)):
            raise ValueError("event arrays differ in length")
        self._E = E
        self._keep = (k, s, v, t, q)
        self._chk(self.lib.fb_tick_launch(self.h, float(now), float(tte), E, _p(k), _p(s), _p(v), _p(t),
                                          _p(q), int(n_pending)))

    def stage(self, now, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None):
        """Validate and stage the next tick's events (host only; overlaps a running tick)."""
        k = _arr(ev_kind, np.uint8)
        s = _arr(ev_slot, np.int32)
        v = _arr(ev_val, np.int32)
        t = _arr(ev_ts, np.float64)
        q = None if ev_seq is None else _arr(ev_seq, np.int64)
        E = len(k)
        if not (len(s) == E and len(v) == E and len(t) == E and (q is None or len(q) == E)):
            raise ValueError("event arrays differ in length")
        self._chk(self.lib.fb_tick_stage(self.h, float(now), E, _p(k), _p(s), _p(v), _p(t), _p(q)))
        self._staged_E = E

    def stage_device(self, now, ev_kind, ev_slot, ev_val, ev_ts, ev_seq=None):
        """Stage a batch already in this GPU's memory (torch tensors on the context's
        device: uint8 / int32 / int32 / float64 / int64): the tick reads it in place and
        its first kernel checks it (an invalid message is overwritten with a harmless one
        and wait() raises naming it).  The tensors must stay unchanged until that tick
        was committed."""
        import torch
        want = ((ev_kind, torch.uint8), (ev_slot, torch.int32), (ev_val, torch.int32), (ev_ts, torch.float64),
                (ev_seq, torch.int64))
        E = int(ev_kind.numel())
        ptrs = []
        for t, dt in want:
            if t is None:
                ptrs.append(None)
                continue
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous() or t.numel() != E:
                raise ValueError("device batch: contiguous %s tensors of %d elements on the GPU expected" % (dt, E))
            dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
            if dev != self.device:
                raise ValueError("device batch on cuda:%d, the context's GPU is cuda:%d" % (dev, self.device))
            ptrs.append(C.c_void_p(t.data_ptr()) if E else None)
        self._chk(self.lib.fb_tick_stage(self.h, float(now), E, *ptrs))
        self._staged_E = E

    def launch_staged(self, tte, n_pending=0):
        """Enqueue the tick on the events of the last stage() (its `now`)."""
        self._chk(self.lib.fb_tick_launch_staged(self.h, float(tte), int(n_pending)))
        self._E = self._staged_E

    def wait(self):
        r = TickResult()
        self._chk(self.lib.fb_tick_wait(self.h, C.byref(r)))
        self.last = r.as_dict()
        return self.last

    def commit(self):
        self._chk(self.lib.fb_tick_commit(self.h))

    def assignments(self, first=0, n=None, out=None):
        """Slot per dispatched task of the waited tick (into ``out`` when given, e.g. a
        ``pinned()`` array)."""
        n = self.last["n_assigned"] - first if n is None else n
        if out is None:
            out = np.zeros(max(n, 1), np.int32)
        elif len(out) < n or out.dtype != np.int32:
            raise ValueError("out must be an int32 array of at least %d entries" % n)
        self._chk(self.lib.fb_get_assignments(self.h, int(first), int(n), out.ctypes.data_as(C.c_void_p)))
        return out[:n]

    def outputs(self, assign=None, orphans=None, evicted=None):
        """The waited tick's assignments, orphans and evicted slots into the given
        arrays (int32 / int64 / int32, e.g. ``pinned()`` ones; None skips a list) with
        one synchronisation; returns the filled views."""
        r = self.last
        for a, n, dt in ((assign, r["n_assigned"], np.int32), (orphans, r["n_orphans_local"], np.int64),
                         (evicted, r["n_evicted"], np.int32)):
            if a is not None and (len(a) < n or a.dtype != dt or not a.flags["C_CONTIGUOUS"]):
                raise ValueError("output array too small or of the wrong type")
        self._chk(self.lib.fb_get_outputs(self.h, None if assign is None else _p(assign),
                                          None if orphans is None else _p(orphans),
                                          None if evicted is None else _p(evicted)))
        return (None if assign is None else assign[: r["n_assigned"]],
                None if orphans is None else orphans[: r["n_orphans_local"]],
                None if evicted is None else evicted[: r["n_evicted"]])

    def set_eager_commit(self, on=True):
        """Eager commits (fb_set_eager_commit): a window tick commits on the device right
        behind itself; wait() and commit() are still called before the next launch."""
        self._chk(self.lib.fb_set_eager_commit(self.h, 1 if on else 0))

    def set_window(self, mode=1):
        """Window ticks (fb_set_window): -1 auto (contexts of more than 128K workers), 0 off,
        1 whenever the last tick was at fill level 0.  Results are identical either way."""
        self._chk(self.lib.fb_set_window(self.h, int(mode)))

    def window_stats(self):
        """(committed window ticks, launches that fell back to the general path)."""
        a, b = C.c_int64(0), C.c_int64(0)
        self._chk(self.lib.fb_window_stats(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def set_compact_out(self, slot, c, orphans, evicted):
        """Register pinned arrays (``pinned()``) that fused ticks fill with their compact
        outputs while they run (fb_set_compact_out); ``outputs_compact`` into the same
        arrays then copies nothing.  A tick uses them only if they fit its worst case --
        slot / c: the queue + 2 x messages positions, orphans: the whole in-flight log,
        evicted: every worker -- and copies otherwise.  ``slot=None`` unregisters."""
        if slot is None:
            self._chk(self.lib.fb_set_compact_out(self.h, None, None, 0, None, 0, None, 0))
            self._cout = self._cout_args = None
            return
        if slot.dtype != np.int32 or c.dtype != np.uint8 or orphans.dtype != np.int64 or evicted.dtype != np.int32:
            raise ValueError("slot int32, c uint8, orphans int64, evicted int32")
        self._chk(self.lib.fb_set_compact_out(self.h, _p(slot), _p(c), min(len(slot), len(c)), _p(orphans),
                                              len(orphans), _p(evicted), len(evicted)))
        self._cout = (slot, c, orphans, evicted)  # keep them alive while registered
        self._cout_args = (_p(slot), _p(c), min(len(slot), len(c)), _p(orphans), _p(evicted))

    def set_compact(self, on=True):
        """Ticks launched afterwards also write the compact assignment form (slot and
        min(c, L + 1) per LRU position): ``outputs_compact`` then reads 5 bytes per
        queued worker instead of 4 per task."""
        self._chk(self.lib.fb_set_compact(self.h, 1 if on else 0))

    def outputs_compact(self, slot, c, orphans=None, evicted=None):
        """The waited tick's compact assignments into ``slot`` (int32) / ``c`` (uint8),
        plus orphans and evicted slots, one synchronisation; returns the filled views
        (slot, c, orphans, evicted).  ``expand(slot, c)`` gives the per-task slots."""
        r = self.last
        cout = getattr(self, "_cout", None)
        if cout is not None and slot is cout[0] and c is cout[1] and orphans is cout[2] and evicted is cout[3]:
            # the registered arrays (the tick wrote them): one call, pointers made at registration
            p0, p1, cap, p2, p3 = self._cout_args
            n = C.c_int64()
            self._chk(self.lib.fb_get_outputs_compact(self.h, p0, p1, cap, C.byref(n), p2, p3))
            return slot[: n.value], c[: n.value], orphans[: r["n_orphans_local"]], evicted[: r["n_evicted"]]
        for a, n, dt in ((orphans, r["n_orphans_local"], np.int64), (evicted, r["n_evicted"], np.int32)):
            if a is not None and (len(a) < n or a.dtype != dt):
                raise ValueError("output array too small or of the wrong type")
        if slot.dtype != np.int32 or c.dtype != np.uint8 or len(c) < len(slot):
            raise ValueError("slot must be int32, c uint8 of at least as many entries")
        n = C.c_int64()
        self._chk(self.lib.fb_get_outputs_compact(self.h, _p(slot), _p(c), len(slot), C.byref(n),
                                                  None if orphans is None else _p(orphans),
                                                  None if evicted is None else _p(evicted)))
        return (slot[: n.value], c[: n.value], None if orphans is None else orphans[: r["n_orphans_local"]],
                None if evicted is None else evicted[: r["n_evicted"]])

    def expand(self, slot, c, out=None):
        """Per-task slots (``assignments()``) from the compact form (host, parallel)."""
        n = self.last["n_assigned"]
        if out is None:
            out = np.zeros(max(n, 1), np.int32)
        slot = np.ascontiguousarray(slot, np.int32)
        c = np.ascontiguousarray(c, np.uint8)
        self._chk(self.lib.fb_expand_compact(self.h, _p(slot), _p(c), len(slot), out.ctypes.data_as(C.c_void_p)))
        return out[:n]

    def local_assignments(self, first=0, n=None):
        """(task index, slot) of the tasks given to this context's workers."""
        n = self.last["n_local"] - first if n is None else n
        task = np.zeros(max(n, 1), np.int64)
        slot = np.zeros(max(n, 1), np.int32)
        self._chk(self.lib.fb_get_local_assignments(self.h, int(first), int(n), _p(task), _p(slot)))
        return task[:n], slot[:n]

    def orphans(self):
        n = self.last["n_orphans_local"]
        out = np.zeros(max(n, 1), np.int64)
        self._chk(self.lib.fb_get_orphans(self.h, int(n), _p(out)))
        return out[:n]

    def evicted(self):
        n = self.last["n_evicted"]
        out = np.zeros(max(n, 1), np.int32)
        self._chk(self.lib.fb_get_evicted(self.h, int(n), _p(out)))
        return out[:n]

    def event_status(self):
        out = np.zeros(max(self._E, 1), np.uint8)
        self._chk(self.lib.fb_get_event_status(self.h, int(self._E), _p(out)))
        return out[: self._E]

    def purge(self, now, tte, commit=True):
        """``purge_workers`` (``task_dispatcher.py:241-249``) alone: expired records
        deleted, the dead registrations' in-flight tasks reported as orphans but not
        dispatched.  Returns dict(result, evicted, orphans)."""
        self._E = 0
        self._chk(self.lib.fb_purge_launch(self.h, float(now), float(tte)))
        res = self.wait()
        out = dict(result=res, evicted=self.evicted(), orphans=self.orphans())
        if commit:
            self.commit()
        return out

    def _pinned_out(self):
        """Reusable pinned output arrays sized for the waited tick (grown geometrically)."""
        r = self.last
        need = (r["n_assigned"], r["n_orphans_local"], r["n_evicted"])
        have = getattr(self, "_pout", None)
        if have is None or any(len(b) < n for b, n in zip(have, need)):
            old = have or (np.zeros(0, np.int32),) * 3
            self._pout = tuple(self.pinned(max(n, 2 * len(b), 1024), dt) for b, n, dt in
                               zip(old, need, (np.int32, np.int64, np.int32)))
        return self._pout

    def _compact_out(self):
        """Registered pinned arrays for the compact outputs (set_compact_out), made once:
        slot / c for the queue plus twice the messages, the orphans for the whole log (up
        to 1M entries; a tick with a longer log copies into them instead), every worker."""
        if getattr(self, "_cbufs", None) is None:
            q = self.max_workers + 2 * self.max_events + 16
            ocap = min(int(self.max_log), 1 << 20)
            self._cbufs = (self.pinned(q, np.int32), self.pinned(q, np.uint8), self.pinned(max(ocap, 1), np.int64),
                           self.pinned(max(self.max_workers, 1), np.int32))
            self.set_compact(True)
            self.set_compact_out(*self._cbufs)
        return self._cbufs

    def tick(self, now, tte, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None, n_pending=0,
             commit=True, outputs=True, pinned=False, compact=False):
        """One full tick.  Returns dict(result, reconnect, assign, orphans, evicted).
        ``pinned=True``: the three lists come back in one readback into reusable pinned
        arrays -- views valid until the next tick.  ``compact=True`` (the drop-in
        dispatcher's path, heartbeat loop): the tick writes slot + min(c, L + 1) per LRU
        position into registered pinned arrays and ``assign`` is a ``CompactAssignments``
        that expands round by round as it is iterated (views valid until the next tick)."""
        if compact and self.mode == "heartbeat":
            bufs = self._compact_out()
        else:
            compact = False
        self.launch(now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, n_pending)
        res = self.wait()
        out = dict(result=res)
        if outputs and compact and res["fill_level"] + 1 > 255:
            compact, pinned = False, True  # rounds beyond a byte: the per-task readback
        if outputs and compact:
            ob = bufs[2]
            if res["n_orphans_local"] > len(ob):  # more orphans than the registered array holds
                ob = np.zeros(res["n_orphans_local"], np.int64)
            sl, cc, o, e = self.outputs_compact(bufs[0], bufs[1], ob, bufs[3])
            out.update(reconnect=self.event_status(), assign=CompactAssignments(sl, cc, res["n_assigned"]),
                       orphans=o, evicted=e)
        elif outputs and pinned:
            a, o, e = self.outputs(*self._pinned_out())
            out.update(reconnect=self.event_status(), assign=a, orphans=o, evicted=e)
        elif outputs:
            out.update(reconnect=self.event_status(), assign=self.assignments(), orphans=self.orphans(),
                       evicted=self.evicted())
        if commit:
            self.commit()
        return out

    # ---------------------------------------------------------------- timing
    def set_stream(self, stream_handle):
        """Run on another HIP stream (an int handle, e.g. torch's cuda_stream), or 0 for the own one."""
        self._chk(self.lib.fb_set_stream(self.h, C.c_void_p(int(stream_handle)) if stream_handle else None))

    def sync(self):
        self._chk(self.lib.fb_sync(self.h))

    def timing_enable(self, on=True):
        self._chk(self.lib.fb_timing_enable(self.h, 1 if on else 0))

    def timing_read(self, max_kernels=32):
        names = (C.c_char_p * max_kernels)()
        ms = (C.c_double * max_kernels)()
        cnt = (C.c_int64 * max_kernels)()
        n = C.c_int32()
        self._chk(self.lib.fb_timing_read(self.h, max_kernels, names, ms, cnt, C.byref(n)))
        return {names[i].decode(): (ms[i], cnt[i]) for i in range(n.value)}

    def timing_gate(self, hold):
        """hold=True: hold the stream (launches queue up behind a gate kernel); False: release.
        Measurement only: the gated launches then run back to back on the device."""
        self._chk(self.lib.fb_timing_gate(self.h, 1 if hold else 0))

    def timing_mark(self):
        """A marker launch (the open gate kernel) that kernel traces can cut a region at."""
        self._chk(self.lib.fb_timing_mark(self.h))

    def timing_span(self):
        """(ms from the gate's end to the release point, gate timed out) after a released gate."""
        ms, to = C.c_double(), C.c_int32()
        self._chk(self.lib.fb_timing_span(self.h, C.byref(ms), C.byref(to)))
        return ms.value, bool(to.value)

    def selftest(self):
        e = C.c_int32()
        self._chk(self.lib.fb_selftest(self.h, C.byref(e)))
        return e.value

    def debug_read(self):
        n = C.c_int64()
        self._chk(self.lib.fb_debug_read(self.h, None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.uint64)
        self._chk(self.lib.fb_debug_read(self.h, _p(out), n.value, C.byref(n)))
        return out[: n.value]

    def device_view(self):
        v = _lib.DeviceView()
        self._chk(self.lib.fb_device_view_get(self.h, C.byref(v)))
        return v
