#!/bin/bash
# SQ instruction-mix counters per kernel for a bench script: tools/pmc_sq.sh <bench.py> <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
B=$R/$1; TAG=$2
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT -o run -- \
    python3 $B --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/err.txt || { tail -5 $OUT/err.txt; exit 5; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for row in csv.DictReader(open(f)):
    k = row["Kernel_Name"].split("(")[0].replace("fb::", "")
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    if row["Counter_Name"] == "SQ_WAVES": n[k] += 1
for k, d in acc.items():
    print(k, "launches", n[k], {c: round(v / max(n[k], 1)) for c, v in sorted(d.items())})
PY
