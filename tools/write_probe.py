"""Diagnostic: k_emit2's HBM write bytes per output array at configs[2].

Builds (here, `--build`) library variants with -DFAASBAL_DIAG_NOW=<mask>, each dropping
the stores of some output arrays (faasbal_kernels.hip: kDiagNow); on the GPU box,
`--run --lib PATH` relaunches the uncommitted configs[2] tick (same input every launch)
so a `rocprofv3 --pmc WRITE_SIZE` pass of each variant gives the bytes that array's
stores cost.  `--summary DIR` prints WRITE_SIZE per k_emit2 launch per variant.

    python tools/write_probe.py --build
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/wp_<m> -o run -- python3 tools/write_probe.py --run --mask <m>
    python tools/write_probe.py --summary gpurun_out
"""
import argparse
import collections
import csv
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-faas_amd"))

MASKS = (0, 1, 3, 4, 8, 16, 32)
WHAT = {0: "all stores", 1: "no trash rows", 3: "no full-round tasks, no trash", 4: "no next free counts",
        8: "no next queue", 16: "no orphans", 32: "no round-L tasks"}


def lib_for(m):
    from faasbal.build import HERE
    return os.path.join(HERE, "libfaasbal_diag%d.so" % m)


def build():
    from faasbal.build import build_lib
    for m in MASKS:
        build_lib(out=lib_for(m), defines=["FAASBAL_DIAG_NOW=%d" % m])
        print("built", lib_for(m))


def run(mask, reps):
    from faasbal import synth
    from faasbal.balancer import GpuBalancer
    st = synth.zipf_state(W=65536, seed=0)
    T = 1_000_000
    g = GpuBalancer(65536, 2 * len(st["log"]) + 2 * T + 65536, max_events=1, lib_path=lib_for(mask))
    g.load(st)
    for _ in range(reps):
        g.launch(1000.0, 10.0, n_pending=T)
        g.wait()
    print("mask %d: %d uncommitted ticks" % (mask, reps))


def summary(d):
    base = None
    for m in MASKS:
        f = glob.glob(os.path.join(d, "wp_%d" % m, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        acc, n = collections.defaultdict(float), collections.Counter()
        for row in csv.DictReader(open(f[0])):
            if row["Counter_Name"] != "WRITE_SIZE":
                continue
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("fb::", "")
            if "k_emit2" in k:
                acc[k] += float(row["Counter_Value"])
                n[k] += 1
        for k in acc:
            kib = acc[k] / n[k]
            base = kib if m == 0 else base
            d_mb = "" if base is None or m == 0 else "  (%+.3f MB)" % ((kib - base) * 1024 / 1e6)
            print("mask %2d %-30s %-24s %4d launches  WRITE %.3f MB%s" % (m, WHAT[m], k[:24], n[k], kib * 1024 / 1e6, d_mb))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--mask", type=int, default=0)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--summary", default="")
    a = ap.parse_args()
    if a.build:
        build()
    if a.run:
        run(a.mask, a.reps)
    if a.summary:
        summary(a.summary)


if __name__ == "__main__":
    main()
