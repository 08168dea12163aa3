#!/bin/bash
# configs[2] host_observed loop: the probe's host split, then its kernel / copy / HIP API
# trace summarised per tick (anchor k_scan).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ho}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python3 -u $R/tools/hostobs_probe.py > $OUT/probe_plain.log 2>&1 || { tail -20 $OUT/probe_plain.log; exit 10; }
cat $OUT/probe_plain.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/trace -o run -- \
    python3 -u $R/tools/hostobs_probe.py > $OUT/probe.log 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 11; }
python3 $R/tools/timeline.py $OUT/trace k_scan > $OUT/timeline.txt || exit 12
cat $OUT/timeline.txt
