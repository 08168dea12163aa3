#!/bin/bash
# Profile pass of the driver's own bench command (python3 bench.py --gpus 1 --steps 20
# --warmup 5, extra arguments appended): kernel-trace stats, then one PMC pass each for
# FETCH_SIZE and WRITE_SIZE (separate runs; no tracing domain beside --pmc).
#   bash tools/prof_driver.sh TAG [bench args]
# Summary into profiles/: python tools/prof_summary.py gpurun_out/prof_TAG TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-drv}
shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $OUT/bench_trace.json 2> $OUT/trace.err || exit 11
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err || exit 12
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/bench_write.json 2> $OUT/write.err || exit 13
