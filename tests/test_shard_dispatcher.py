"""The sharded drop-in: GpuPushDispatcher over a worker table split across ranks
(faasbal.sharded groups; ShardedPushDispatcher), replaying the reference-captured
golden vectors message for message (tests/test_dispatcher.replay_golden).

* CPU: two processes over gloo, each rank's shard computed by the numpy protocol
  model (tests/shard_model_balancer.py) -- rank 0 runs the ZMQ/Redis loop,
  broadcasts every call, gathers the per-rank (task, slot) pairs.
* GPU, one process: LocalShardGroup of ShardedBalancer contexts (the exchange
  summed on the device).
* GPU, two processes over RCCL (skipped below two GPUs).
"""
import glob
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = sorted(p for p in glob.glob(os.path.join(HERE, "golden", "*.npz"))
                if not os.path.basename(p).startswith("deque_"))
# the small adversarial vectors, the configs[1]/[2] shapes and the churn stream
SUBSET = [p for p in GOLDEN if os.path.basename(p)[:-4] in
          ("small_%02d" % i for i in range(0, 48, 3))] + \
         [p for p in GOLDEN if os.path.basename(p).startswith("cfg")]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, backend, paths, errq):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "distributed-faas_amd"))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from faasbal.dispatcher import ShardedPushDispatcher
    from test_dispatcher import golden_sizes, replay_golden
    if backend == "nccl":
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def backend_balancer(sizes):
        if backend == "gloo":
            from shard_model_balancer import ModelRankBalancer
            return ModelRankBalancer(rank, world, sizes["max_workers"])
        return None  # ShardedBalancer on this rank's GPU

    try:
        for path in paths:
            z = np.load(path)
            sizes = golden_sizes(z)
            if rank == 0:
                def make(sz, env, z=z):
                    return ShardedPushDispatcher("127.0.0.1", 0, float(z["tte"]), **sz, redis_client=env,
                                                 subscriber=env, socket=env, poller=env, clock=env.clock,
                                                 backend_balancer=backend_balancer(sz), device=rank)
                d = None
                try:
                    d = replay_golden(z, make)
                finally:
                    if d is not None:
                        d.balancer.close()
            else:
                ShardedPushDispatcher("127.0.0.1", 0, float(z["tte"]), **sizes,
                                      backend_balancer=backend_balancer(sizes), device=rank)
    except Exception as e:  # report to the parent, keep the peer from hanging
        errq.put("rank %d: %r" % (rank, e))
        raise
    finally:
        dist.destroy_process_group()


def _spawn(world, backend, paths, timeout=600):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, backend, paths, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_sharded_dispatcher_gloo_world2_replays_reference():
    _spawn(2, "gloo", SUBSET)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_dispatcher_one_gpu_replays_reference(world):
    sys.path.insert(0, HERE)
    from faasbal.dispatcher import GpuPushDispatcher
    from faasbal.sharded import LocalShardGroup
    from test_dispatcher import replay_golden
    for path in GOLDEN:
        z = np.load(path)

        def make(sz, env, z=z):
            group = LocalShardGroup(world, sz["max_workers"], sz["max_inflight"], max_events=sz["max_events"])
            return GpuPushDispatcher("127.0.0.1", 0, float(z["tte"]), **sz, redis_client=env, subscriber=env,
                                     socket=env, poller=env, clock=env.clock, balancer=group)
        d = replay_golden(z, make)
        d.balancer.close()


@pytest.mark.gpu
def test_sharded_dispatcher_rccl_world2_replays_reference():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (one process per GPU over RCCL)")
    _spawn(2, "nccl", SUBSET)


def _fail_rank_main(rank, world, port, errq):
    """DistShardGroup when a tick fails on one rank only: the failure
    reaches rank 0 as the FaasbalError, no rank commits that tick, and the group keeps
    serving (no rank left blocked in a collective)."""
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "distributed-faas_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from faasbal import synth
    from faasbal._lib import FB_ENOSPC, FaasbalError
    from faasbal.sharded import DistShardGroup, serve_shard
    from shard_model_balancer import ModelRankBalancer
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class Flaky(ModelRankBalancer):
        """Rank 1's balancer fails its second tick after the exchange (as an in-flight
        log shard that is full would: FB_ENOSPC from fb_tick_wait)."""
        n = 0

        def tick(self, *a, **k):
            out = super().tick(*a, **k)
            Flaky.n += 1
            if rank == 1 and Flaky.n == 2:
                raise FaasbalError(FB_ENOSPC, "log shard full (injected)")
            return out

    try:
        st = synth.zipf_state(W=64, seed=3)
        bal = Flaky(rank, world, 64)
        if rank != 0:
            serve_shard(bal)
            return
        g = DistShardGroup(bal, 64)
        g.load(st)
        g.tick(1000.0, 10.0, n_pending=40)
        before = g.read_state()
        try:
            g.tick(1000.5, 10.0, n_pending=40)
            raise AssertionError("the failing rank's error did not reach rank 0")
        except FaasbalError as e:
            assert e.code == FB_ENOSPC, e
        after = g.read_state()  # the group still serves; nothing was committed
        for key in ("reg", "free", "queue", "log"):
            assert np.array_equal(before[key], after[key]), key
        assert after["head"] == before["head"]
        g.tick(1000.5, 10.0, n_pending=40)  # and ticks again
        g.close()
    except Exception as e:
        errq.put("rank %d: %r" % (rank, e))
        raise
    finally:
        dist.destroy_process_group()


def test_dist_shard_group_survives_a_failing_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_fail_rank_main, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
