#!/bin/bash
# Round-3 measurement pass on the GPU box: configs[2] kernel stats + PMC (tools/prof_pmc.sh),
# in-kernel stamps of configs[2], the configs[4]-per-GPU stream line.  Each step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-r03}
bash tools/prof_pmc.sh ${TAG}_c2 > gpurun_out/${TAG}_c2_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_c2_pmc.log; exit 1; }
cd $R
timeout -k 10 200 python -u tools/stamps.py > gpurun_out/${TAG}_stamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_stamps.txt; exit 2; }
timeout -k 10 300 python -u bench.py --workload stream > gpurun_out/${TAG}_stream.json 2> gpurun_out/${TAG}_stream.err \
    || { tail -20 gpurun_out/${TAG}_stream.err; exit 3; }
cat gpurun_out/${TAG}_c2_pmc.log | tail -8
cat gpurun_out/${TAG}_stream.json
