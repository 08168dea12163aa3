#!/bin/bash
# Round-3 measurement pass on the GPU box: configs[2] kernel stats + FETCH/WRITE PMC passes
# (tools_profile.sh), in-kernel stamps of configs[2], a kernel trace of the stream line.
# Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-r03}
bash tools_profile.sh ${TAG}_c2 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
cd $R
timeout -k 10 200 python -u tools/stamps.py > gpurun_out/${TAG}_stamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_stamps.txt; exit 2; }
OUT=$R/gpurun_out/prof_${TAG}_stream
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --workload stream > $OUT/bench_trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 3; }
cat $R/gpurun_out/prof_${TAG}_c2/bench_trace.json
cat $OUT/bench_trace.json
