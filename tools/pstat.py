"""Print a rocprofv3 kernel_stats.csv (name, calls, average us) for each directory given."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    print("==", d)
    for r in csv.DictReader(open(f[0])):
        print("  %-44s %5s %9.2f us" % (r["Name"][:44], r["Calls"], float(r["AverageNs"]) / 1e3))
