"""Summarise a tools_profile.sh run into profiles/ (tracked).

    python tools/prof_summary.py gpurun_out/prof_<tag> <tag>

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats),
profiles/<tag>_kernel_modal.csv (per kernel, the launches of its most frequent grid
size: the bench's own tick, without the other states the run also launches),
profiles/<tag>_kernel_timed.csv (the launches of the bench's timed region, cut at the
two marker launches bench.py places around it, and of its gated per-kernel timing pass),
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
                vals[(short(r["Kernel_Name"]), ctr)].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    kernels = sorted({k for k, _ in vals})
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = float(r["AverageNs"])
    # the benchmark's own tick among the others the run launches (committed_tick's depleted
    # states, the host paths' readback kernels): per kernel, the launches of its most frequent
    # grid size -- the timed, gated and host-observed ticks of the bench's state
    trace = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
        trace[short(r["Kernel_Name"])][int(r["Grid_Size_X"])].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    modal = {}
    for k, byg in trace.items():
        grid, ds = max(byg.items(), key=lambda kv: len(kv[1]))
        ds = sorted(ds)
        modal[k] = dict(grid=grid, launches=len(ds), avg_ns=sum(ds) / len(ds), median_ns=ds[len(ds) // 2])
    with open(os.path.join(prof, "%s_kernel_modal.csv" % tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid", "launches", "avg_ns", "median_ns", "all_launches_avg_ns"])
        for k in sorted(modal):
            m = modal[k]
            w.writerow([k, m["grid"], m["launches"], "%.0f" % m["avg_ns"], m["median_ns"], "%.0f" % stats.get(k, 0)])
    # bench.py's regions, cut at its gate-kernel launches: the two markers bracket the timed
    # (host-paced) steps; the next gate holds the K steps of the per-kernel timing pass
    # (gated_timing: back to back on the device), up to the gate after it
    rows = sorted(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))),
                  key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    gates = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "gate"]
    # (a marker opens at once, ~3 us; a held gate waits for the host's enqueue of its batch)
    marks = [i for i in gates if dur(rows[i]) < 10000]
    timed, gated = {}, {}
    regions = []
    if len(marks) >= 2:
        regions.append(("timed", timed, marks[0], marks[1]))
    if len(marks) >= 3:
        # from the first held gate after the second marker to the third marker
        held = [i for i in gates if marks[1] < i < marks[2]]
        if held:
            regions.append(("gated", gated, held[0], marks[2]))
    with open(os.path.join(prof, "%s_kernel_timed.csv" % tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["region", "kernel", "launches", "avg_ns", "min_ns", "max_ns", "region_span_ns"])
        for name, dst, i0, i1 in regions:
            per = collections.defaultdict(list)
            for r in rows[i0 + 1:i1]:
                if short(r["Kernel_Name"]) != "gate":
                    per[short(r["Kernel_Name"])].append(dur(r))
            span = int(rows[i1 - 1]["End_Timestamp"]) - int(rows[i0 + 1]["Start_Timestamp"])
            for k in sorted(per):
                ds = per[k]
                dst[k] = sum(ds) / len(ds)
                w.writerow([name, k, len(ds), "%.0f" % dst[k], min(ds), max(ds), span])
    # PMC passes: the same restriction (the counter rows carry the grid size)
    pmc_grid = {k: m["grid"] for k, m in modal.items()}
    with open(os.path.join(prof, "%s_pmc.csv" % tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "launches", "FETCH_SIZE_KiB_avg", "WRITE_SIZE_KiB_avg", "hbm_bytes_per_launch",
                    "trace_avg_ns"])
        out = {}
        for k in kernels:
            def sel(ctr):
                v = vals.get((k, ctr), [])
                g = [x for gr, x in v if gr == pmc_grid.get(k, gr)]
                return g or [x for _, x in v] or [0.0]
            fe, wr = sel("FETCH_SIZE"), sel("WRITE_SIZE")
            fa, wa = sum(fe) / len(fe), sum(wr) / len(wr)
            b = (2 * fa + wa) * 1024
            m = modal.get(k, {})
            w.writerow([k, len(fe), "%.1f" % fa, "%.1f" % wa, int(b), "%.0f" % stats.get(k, 0)])
            out[k] = dict(fetch_kib=fa, write_kib=wa, hbm_bytes=b, trace_avg_ns=stats.get(k),
                          trace_modal_avg_ns=m.get("avg_ns"), trace_modal_median_ns=m.get("median_ns"),
                          trace_modal_grid=m.get("grid"), trace_timed_avg_ns=timed.get(k),
                          trace_gated_avg_ns=gated.get(k))
    bench = json.loads(open(os.path.join(d, "bench_trace.json")).read().strip().splitlines()[-1])
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
