"""Summarise a tools_profile.sh run into profiles/ (tracked).

    python tools/prof_summary.py gpurun_out/prof_<tag> <tag>

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats),
profiles/<tag>_pmc.csv (per-kernel average FETCH_SIZE / WRITE_SIZE per launch,
KiB) and profiles/traffic.json, which bench.py reports as roofline.traffic:
HBM-side bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (the gfx950 FETCH_SIZE
halving, /opt/skills/guides/MI355X_MICROARCH.md "HBM").
"""
import collections
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """Kernel symbol -> the timer name bench.py reports (k_emit2 is the fused 'emit')."""
    n = name.split("(")[0].split("<")[0].split("::")[-1].replace("k_", "", 1)
    return "emit" if n == "emit2" else n


def main(d, tag):
    prof = os.path.join(REPO, "profiles")
    shutil.copy(os.path.join(d, "trace", "run_kernel_stats.csv"), os.path.join(prof, "%s_kernel_stats.csv" % tag))
    vals = collections.defaultdict(list)
    for sub, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        for r in csv.DictReader(open(os.path.join(d, sub, "run_counter_collection.csv"))):
            if r["Counter_Name"] == ctr:
                vals[(short(r["Kernel_Name"]), ctr)].append(float(r["Counter_Value"]))
    kernels = sorted({k for k, _ in vals})
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = float(r["AverageNs"])
    with open(os.path.join(prof, "%s_pmc.csv" % tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "launches", "FETCH_SIZE_KiB_avg", "WRITE_SIZE_KiB_avg", "hbm_bytes_per_launch",
                    "trace_avg_ns"])
        out = {}
        for k in kernels:
            fe = vals.get((k, "FETCH_SIZE"), [0.0])
            wr = vals.get((k, "WRITE_SIZE"), [0.0])
            fa, wa = sum(fe) / len(fe), sum(wr) / len(wr)
            b = (2 * fa + wa) * 1024
            w.writerow([k, len(fe), "%.1f" % fa, "%.1f" % wa, int(b), "%.0f" % stats.get(k, 0)])
            out[k] = dict(fetch_kib=fa, write_kib=wa, hbm_bytes=b, trace_avg_ns=stats.get(k))
    bench = json.load(open(os.path.join(d, "bench_trace.json")))
    cfg = bench["config"]
    traffic = dict(tag=tag, workers=cfg["workers"], tasks_per_tick=cfg["tasks_per_tick"], n_gpus=bench["n_gpus"],
                   kernels=out, note="HBM-side bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KiB->B), "
                                     "rocprofv3 --pmc passes of bench.py, profiles/%s_pmc.csv; trace_avg_ns from "
                                     "profiles/%s_kernel_stats.csv" % (tag, tag))
    json.dump(traffic, open(os.path.join(prof, "%s_traffic.json" % tag), "w"), indent=1)
    # profiles/traffic.json: the latest summary per configuration (bench.py looks its own up)
    tp = os.path.join(prof, "traffic.json")
    allt = json.load(open(tp)) if os.path.exists(tp) else {}
    if "entries" not in allt:
        allt = {"entries": {}}
    # (the streaming bench's entries carry a "stream," prefix: same workers and tasks, other kernels)
    pre = "stream," if "events_per_tick" in cfg else ""
    allt["entries"]["%s%d,%d,%d" % (pre, traffic["workers"], traffic["tasks_per_tick"], traffic["n_gpus"])] = traffic
    json.dump(allt, open(tp, "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
