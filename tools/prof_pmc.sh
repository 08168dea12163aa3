#!/bin/bash
# rocprof kernel stats + FETCH_SIZE / WRITE_SIZE passes (one counter group per pass) of a
# bench.py run: tools/prof_pmc.sh TAG [bench args].  Summary: tools/pmc_summary.py gpurun_out/pmc_TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-host-observed "$@" > $OUT/bench_trace.json 2> $OUT/trace.err || exit 11
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-host-observed "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err || exit 12
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-host-observed "$@" > $OUT/bench_write.json 2> $OUT/write.err || exit 13
python3 $R/tools/pmc_summary.py $OUT
