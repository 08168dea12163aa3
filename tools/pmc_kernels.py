"""Per-kernel averages of every counter in a rocprofv3 --pmc directory (plus the
kernel trace's average duration when present): python3 tools/pmc_kernels.py DIR"""
import collections
import csv
import glob
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(lambda: collections.Counter())
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("fb::", "")
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            n[k][row["Counter_Name"]] += 1
    dur = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("fb::", "")
            dur[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    print("==", d)
    for k in sorted(acc):
        ds = dur.get(k, [])
        avg = sum(ds) / len(ds) / 1e3 if ds else float("nan")
        cs = " ".join("%s=%.0f" % (c.replace("TCP_UTCL1_", "").replace("TCP_TCC_", "").replace("SQ_", "").replace("_sum", ""), acc[k][c] / n[k][c])
                      for c in sorted(acc[k]))
        print("%-28s %6.1f us  %s" % (k[:28], avg, cs))


if __name__ == "__main__":
    main(sys.argv[1])
