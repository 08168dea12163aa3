#!/bin/bash
# configs[3] on one GPU (16M tasks x 1M workers): bench line, kernel stats and FETCH/WRITE
# PMC passes (tools/prof_pmc.sh).  Each step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-c3}
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --steps 50 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
bash tools/prof_pmc.sh ${TAG} --workload cfg3 --steps 30 --warmup 3 > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 2; }
cat gpurun_out/${TAG}_pmc.log
