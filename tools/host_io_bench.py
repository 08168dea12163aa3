"""Host I/O of the drop-in dispatcher per tick, on the GPU box.

GpuPushDispatcher with the real HIP balancer and in-memory transports: a Redis
client whose every round trip costs a simulated RTT (busy wait; a localhost
Redis answers in tens of microseconds), a ROUTER socket that counts frames.
Per tick: N registered workers, T new tasks.  Compares the reference's
per-command I/O (3 round trips per task) with the pipelined tick (2 per tick)
and times the codec (dill vs the C-pickler path, byte-identical output).

    python tools/host_io_bench.py [--workers 4096 --tasks 20000 --rtt-us 50 --ticks 3]
"""
import argparse
import collections
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))

from faasbal import codec  # noqa: E402
from faasbal.dispatcher import GpuPushDispatcher  # noqa: E402


def spin(us):
    t = time.perf_counter() + us * 1e-6
    while time.perf_counter() < t:
        pass


class Pipe:
    def __init__(self, env):
        self.env, self.cmds = env, []

    def hget(self, key, field):
        self.cmds.append((key, field))

    def hset(self, key, mapping=None):
        self.cmds.append(None)

    def execute(self):
        self.env.trip()
        out = [("%s:%s" % (c[1], c[0])).encode() if c is not None else 1 for c in self.cmds]
        self.cmds = []
        return out


class Env:
    def __init__(self, rtt_us, pipelines):
        self.rtt_us, self.trips, self.frames = rtt_us, 0, 0
        self.inbound, self.tasks = collections.deque(), collections.deque()
        if pipelines:
            self.pipeline = lambda transaction=True: Pipe(self)

    def trip(self):
        self.trips += 1
        spin(self.rtt_us)

    def poll(self, timeout=None):
        return [(self, 1)] if self.inbound else []

    def recv_multipart(self):
        w, frame = self.inbound.popleft()
        return [w, frame]

    def send_multipart(self, parts):
        self.frames += 1

    def get_message(self):
        return {"type": "message", "data": self.tasks.popleft().encode()} if self.tasks else None

    def hget(self, key, field):
        self.trip()
        return ("%s:%s" % (field, key)).encode()

    def hset(self, key, mapping=None):
        self.trip()


def run(args, pipelines):
    env = Env(args.rtt_us, pipelines)
    d = GpuPushDispatcher("127.0.0.1", 0, 1e9, max_workers=args.workers, max_events=args.workers + 16,
                          max_inflight=args.tasks * (args.ticks + 2) + 16, redis_client=env, subscriber=env,
                          socket=env, poller=env, batch_io=pipelines)
    per = -(-args.tasks * (args.ticks + 1) // args.workers)
    for w in range(args.workers):
        env.inbound.append((b"w%06d" % w, codec.serialize({"type": "register",
                                                            "data": {"num_processes": per}}).encode()))
    d.tick()  # registrations
    times, trips = [], []
    for t in range(args.ticks):
        env.tasks.extend("t%d_%d" % (t, j) for j in range(args.tasks))
        t0, n0 = time.perf_counter(), env.trips
        d.tick()
        times.append(time.perf_counter() - t0)
        trips.append(env.trips - n0)
    return min(times), trips[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4096)
    ap.add_argument("--tasks", type=int, default=20000)
    ap.add_argument("--rtt-us", type=float, default=50.0)
    ap.add_argument("--ticks", type=int, default=3)
    args = ap.parse_args()
    per_call, trips_a = run(args, False)
    batched, trips_b = run(args, True)
    import dill
    m = {"type": "task", "data": {"task_id": "0f8fad5b-d9cb-469f-a165-70867728950e", "fn_payload": "gASV" * 60,
                                  "param_payload": "gAS" * 30}}
    n = 20000
    t0 = time.perf_counter()
    for _ in range(n):
        __import__("codecs").encode(dill.dumps(m), "base64").decode()
    t1 = time.perf_counter()
    for _ in range(n):
        codec.serialize(m)
    t2 = time.perf_counter()
    print(json.dumps({
        "workload": "one dispatcher tick: %d tasks over %d workers, simulated Redis RTT %.0f us"
                    % (args.tasks, args.workers, args.rtt_us),
        "per_command": {"tick_ms": per_call * 1e3, "redis_round_trips": trips_a,
                        "tasks_per_s": args.tasks / per_call},
        "pipelined": {"tick_ms": batched * 1e3, "redis_round_trips": trips_b, "tasks_per_s": args.tasks / batched},
        "codec_us_per_task_message": {"dill": (t1 - t0) / n * 1e6, "c_pickler": (t2 - t1) / n * 1e6},
    }))


if __name__ == "__main__":
    main()
