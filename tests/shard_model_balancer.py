"""TEST DOUBLE: one rank of a sharded table computed by the numpy protocol model
(tests/shard_model.py) behind ShardedBalancer's per-rank API (load / read_state /
tick / purge with the exchange all-reduce over torch.distributed).  Lets the CPU
suite run faasbal.sharded's groups and the sharded drop-in dispatcher over gloo
without a GPU; the GPU suite runs the same tests on libfaasbal."""
import numpy as np
import torch
import torch.distributed as dist

import shard_model as sm


class ModelRankBalancer:
    def __init__(self, rank, world, n_workers):
        self.rank, self.world, self.W = rank, world, int(n_workers)
        self.rs = None
        self.full_assign = False

    def set_full_assign(self, on=True):
        self.full_assign = bool(on)

    def close(self):
        pass

    def load(self, st):
        self.rs = sm.split(st, self.world, self.rank)

    def read_state(self, with_log=True):
        rs = self.rs
        out = dict(base=rs["base"], reg=rs["reg"].astype(np.uint8), free=rs["free"].astype(np.int32),
                   hb=rs["hb"].astype(np.float64), epoch=rs["epoch"].astype(np.uint32),
                   queue=np.asarray(rs["queue"], np.int32), head=int(rs["head"]))
        if with_log:
            out.update(log=np.asarray(rs["log_slot"], np.int32), log_seq=np.asarray(rs["log_seq"], np.int64))
        return out

    def _exchange(self, x, allreduce):
        xt = torch.from_numpy(x)
        (allreduce or dist.all_reduce)(xt)  # SUM of uint8, one contributor per byte
        return xt.numpy()

    def _run(self, now, tte, k, s, v, t, q, T, allreduce, redist, commit):
        head = int(self.rs["head"])
        x, ctx = sm.phase1(self.rs, self.world, self.rank, now, tte, k, s, v, t, q, T)
        out, self._next = sm.phase2(self.rs, ctx, self._exchange(x, allreduce), redist=redist)
        n = int(out["n_assigned"])
        full = out.pop("assign_all")
        if self.full_assign:
            out["assign"] = full
        out["result"] = dict(n_assigned=n, log_head=head + n, n_local=len(out["task"]),
                             n_orphans_local=len(out["orphans"]), n_evicted=len(out["evicted"]))
        if commit:
            self.commit()
        return out

    def commit(self):
        self.rs = self._next

    def tick(self, now, tte, ev_kind=(), ev_slot=(), ev_val=(), ev_ts=(), ev_seq=None, n_pending=0,
             allreduce=None, commit=True):
        k = np.asarray(ev_kind, np.int64)
        seq = np.full(len(k), -1, np.int64) if ev_seq is None else np.asarray(ev_seq, np.int64)
        return self._run(now, tte, k, np.asarray(ev_slot, np.int64), np.asarray(ev_val, np.int64),
                         np.asarray(ev_ts, np.float64), seq, int(n_pending), allreduce, True, commit)

    def purge(self, now, tte, allreduce=None, commit=True):
        e = np.zeros(0, np.int64)
        out = self._run(now, tte, e, e, e, np.zeros(0), e, 0, allreduce, False, commit)
        return dict(result=out["result"], evicted=out["evicted"], orphans=out["orphans"])
