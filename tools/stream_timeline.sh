#!/bin/bash
# Per-tick device/host timeline of the pipelined streaming tick (tools/stream_probe.py,
# pinned messages): kernel, memory-copy and HIP API traces (no counters), summarised by
# tools/timeline.py into gaps between the tick's kernels and the host calls behind them.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tl}
MODE="${2:---pinned}"
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/trace -o run -- \
    python3 -u $R/tools/stream_probe.py $MODE > $OUT/probe.log 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 11; }
tail -2 $OUT/probe.log
python3 $R/tools/timeline.py $OUT/trace > $OUT/timeline.txt || exit 12
cat $OUT/timeline.txt
