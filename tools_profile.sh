#!/bin/bash
# Profile recipe run on the GPU box: kernel-trace stats, then one PMC
# pass per TCC counter group (FETCH_SIZE / WRITE_SIZE cannot share a pass), of bench.py
# with the given extra arguments:  bash tools_profile.sh TAG [bench args]
# Summary into profiles/: python tools/prof_summary.py gpurun_out/prof_TAG TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-observed "$@" > $OUT/bench_trace.json 2> $OUT/trace.err || exit 11
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-host-observed "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err || exit 12
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-host-observed "$@" > $OUT/bench_write.json 2> $OUT/write.err || exit 13
