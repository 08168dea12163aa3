"""The configs[2] tick's folded commit cost (bench.committed_tick) for the library named
by FAASBAL_LIB (A/B of builds): python tools/commit_probe.py [--reps 20]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))
import bench  # noqa: E402
from faasbal import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--workers", type=int, default=65536)
ap.add_argument("--tasks", type=int, default=1_000_000)
args = ap.parse_args()
st = synth.zipf_state(W=args.workers, seed=0)
cm = bench.committed_tick(st, args.tasks, reps=args.reps)
print(os.path.basename(os.environ.get("FAASBAL_LIB", "in-tree")),
      json.dumps({k: (round(v * 1e3, 2) if isinstance(v, float) else v) for k, v in cm.items()
                  if not isinstance(v, dict)}),
      {k: round(v * 1e3, 2) for k, v in cm["kernels_with_commit_ms"].items()},
      {k: round(v * 1e3, 2) for k, v in cm["kernels_ms"].items()}, flush=True)
