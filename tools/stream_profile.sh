#!/bin/bash
# rocprofv3 kernel-trace stats of the streaming bench (configs[4] per GPU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
OUT=$R/gpurun_out/prof_stream_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --workload stream > $OUT/bench_trace.json 2> $OUT/trace.err || exit 21
find $OUT -name "*stats.csv"
