"""Sharded tick protocol over torch.distributed (gloo, world_size 2) on CPU.

Each rank runs the numpy model of its phases (tests/shard_model.py) on its own
slot range; the exchange buffers are all-reduced with ``dist.all_reduce``
exactly as bench.py / ShardedBalancer do with RCCL on GPUs.  Rank 0 merges the
per-rank outputs and checks them, and the reassembled state, against the
sequential oracle for several multi-tick scenarios.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard_model as sm
from faasbal import synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scenarios():
    out = []
    for seed in range(4):
        W = [37, 300][seed % 2]
        scen = synth.random_scenario(7000 + seed, W=W, n_ticks=4, max_events=[20, 200][seed % 2],
                                     max_new=[50, 400][seed // 2])
        st = dict(reg=scen["init_reg"], free=scen["init_free"], hb=scen["init_hb"], epoch=scen["init_epoch"],
                  queue=scen["init_queue"], log=scen["init_log"])
        out.append(("random%d" % seed, st, scen["tte"], scen["ticks"]))
    st = synth.zipf_state(W=2048, seed=4)
    out.append(("zipf", st, 10.0, [dict(now=1000.0, n_new=30000, ev_kind=np.zeros(0, np.uint8),
                                        ev_slot=np.zeros(0, np.int32), ev_val=np.zeros(0, np.int32),
                                        ev_ts=np.zeros(0), ev_pick=np.zeros(0, np.uint32))]))
    return out


def _worker(rank, world, port, errq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import Oracle

        for name, st, tte, ticks in _scenarios():
            W = len(st["reg"])
            rs = sm.split(st, world, rank)
            o = Oracle(W, len(st["log"]) + 200_000) if rank == 0 else None
            if o is not None:
                o.load(st["reg"], st["free"], st["hb"], st["epoch"], st["queue"], st["log"])
            # result events resolve to sequence numbers from the global log (reassembled from the shards)
            carried = 0
            for t, tk in enumerate(ticks):
                shards = [None] * world
                dist.all_gather_object(shards, (rs["log_seq"], rs["log_slot"], rs["head"]))
                glog = np.full(shards[0][2], -1, np.int64)
                for q, sl, _ in shards:
                    glog[q] = sl
                seq = np.full(len(tk["ev_kind"]), -1, np.int64)
                for i in np.nonzero(tk["ev_kind"] == synth.EV_RESULT)[0]:
                    mine = np.nonzero(glog == tk["ev_slot"][i])[0]
                    if len(mine) and tk["ev_pick"][i] % 5 != 4:
                        seq[i] = mine[tk["ev_pick"][i] % len(mine)]
                T = carried + tk["n_new"]
                args = (tk["now"], tte, tk["ev_kind"], tk["ev_slot"], tk["ev_val"], tk["ev_ts"], seq, T)
                x, ctx = sm.phase1(rs, world, rank, *args)
                xt = torch.from_numpy(x)
                dist.all_reduce(xt)  # SUM of uint8: one nonzero contributor per byte
                out, rs = sm.phase2(rs, ctx, xt.numpy())
                outs = [None] * world
                dist.all_gather_object(outs, out)
                states = [None] * world
                dist.all_gather_object(states, rs)
                if rank == 0:
                    b = o.tick(*args)
                    assign = np.full(out["n_assigned"], -1, np.int32)
                    for u in outs:
                        assign[u["task"]] = u["slot"]
                    np.testing.assert_array_equal(assign, b["assign"], err_msg="%s t%d assign" % (name, t))
                    np.testing.assert_array_equal(np.sort(np.concatenate([u["orphans"] for u in outs])),
                                                  b["orphans"], err_msg="%s t%d orphans" % (name, t))
                    np.testing.assert_array_equal(np.sort(np.concatenate([u["evicted"] for u in outs])),
                                                  b["evicted"], err_msg="%s t%d evicted" % (name, t))
                    np.testing.assert_array_equal(out["reconnect"], b["reconnect"])
                    so = o.export()
                    reg = so["reg"].astype(bool)
                    glog = np.full(len(so["log"]), -1, np.int64)
                    for s2 in states:
                        lo, hi = s2["base"], s2["base"] + s2["n"]
                        np.testing.assert_array_equal(s2["reg"], reg[lo:hi])
                        m = reg[lo:hi]
                        np.testing.assert_array_equal(s2["free"][m], so["free"][lo:hi][m])
                        np.testing.assert_array_equal(s2["hb"][m], so["hb"][lo:hi][m])
                        np.testing.assert_array_equal(s2["queue"], so["queue"])
                        glog[s2["log_seq"]] = s2["log_slot"]
                    np.testing.assert_array_equal(glog, so["log"], err_msg="%s t%d log" % (name, t))
                    carried = T + len(b["orphans"]) - len(b["assign"])
                carried = [carried]
                dist.broadcast_object_list(carried, src=0)
                carried = carried[0]
    except Exception as e:  # report to the parent, keep the peer from hanging
        errq.put("rank %d: %r" % (rank, e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_protocol_gloo_world2():
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
