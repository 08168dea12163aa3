"""TEST DOUBLE: the oracle (oracle/push_oracle.c) behind GpuBalancer's tick API.

Lets the CPU suite exercise GpuPushDispatcher's host logic (identity -> slot
mapping, message decoding, reply/Redis ordering, orphan bookkeeping, log
compaction) without a GPU.  Never imported by the product package; the GPU
suite runs the same tests against the real HIP library.
"""
import numpy as np

from faasbal._lib import FB_ENOSPC, FaasbalError
from oracle import DequeOracle, Oracle


class OracleBalancer:
    def __init__(self, max_workers, max_log, max_events=0, device=0, mode="heartbeat", max_tokens=None):
        self.mode = mode
        self.o = DequeOracle(max_workers, max_log) if mode == "deque" else Oracle(max_workers, max_log)

    def close(self):
        pass

    def load_state(self, reg, free, hb, epoch=None, queue=(), log=()):
        epoch = np.zeros(len(reg), np.uint32) if epoch is None else epoch
        self.o.load(reg, free, hb, epoch, queue, log)

    def read_state(self, with_log=True):
        return self.o.export()

    def tick(self, now, tte, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None, n_pending=0, pinned=False,
             compact=False):
        # (pinned / compact: GpuBalancer's readback forms -- the oracle's outputs are host arrays)
        if ev_seq is None:
            ev_seq = np.full(len(ev_kind), -1, np.int64)
        # the HIP tick fails with FB_ENOSPC and commits nothing when its dispatches do not
        # fit the in-flight log; the oracle stops mid-tick, so its state is restored
        snap = self.o.export() if self.mode != "deque" else None
        try:
            out = self.o.tick(now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, n_pending)
        except RuntimeError as e:
            if snap is None or "overflow" not in str(e):
                raise
            self.o.load(snap["reg"], snap["free"], snap["hb"], snap["epoch"], snap["queue"], snap["log"])
            raise FaasbalError(FB_ENOSPC, "in-flight log full (oracle double)")
        out["result"] = dict(n_assigned=len(out["assign"]), n_orphans=len(out["orphans"]),
                             log_head=self.o.export()["head"])
        return out

    def purge(self, now, tte):
        # purge_workers alone: orphans reported, none dispatched (dispatch_limit = 0)
        out = self.o.tick(now, tte, [], [], [], [], np.zeros(0, np.int64), 0, dispatch_limit=0)
        out["result"] = dict(n_assigned=0, n_orphans=len(out["orphans"]), log_head=self.o.export()["head"])
        return out
