#!/bin/bash
# GPU box: one rocprofv3 --pmc pass (+ kernel trace) of a bench.py run, per-kernel counter averages.
#   PMC="<counters>" tools/pmc_bench.sh TAG [bench args]   -> gpurun_out/pmcb_TAG/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d $R/gpurun_out/pmcb_$T -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-host-observed "$@" > $R/gpurun_out/pmcb_$T.json 2> $R/gpurun_out/pmcb_$T.err || { tail -5 $R/gpurun_out/pmcb_$T.err; exit 1; }
python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmcb_$T
